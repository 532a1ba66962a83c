"""The reference's lexicographic SOR order at any grid size on the GPU
(ordering="lex", small_solve="off" for the cavity: csrc/lexw.hpp, the red-black march with the
i+j time skew), bit for bit against the oracle's restatement of the
reference's own loop (oracle/ ORC_LEX, pinned to the reference binaries by
tests/test_oracle_golden.py).

Bars: iteration counts equal, reported residual equal, every field equal bit
for bit — at capped sweep counts where the solve runs into the cap (the
BASELINE sizes), at converging solves (the early stop and its replay), on
1..3 strips, for 1 to 4 sweeps per launch (4, the default on one strip,
with 110-column tiles: lexw.hpp lexw_twc; widths 219/220 put the last
columns on a 110-column tile edge).
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LEXW = {"resident": 0}  # the multi-block march (the resident launch has its own tests: test_gpu_resident.py)

import cfd_amd as C  # noqa: E402
import oracle as O  # noqa: E402
from test_gpu_parity import assert_bits, ofield  # noqa: E402


def solve_both(cp, f, strips=1, spl=0):
    g = C.CavitySolver(cp, ordering="lex", small_solve="off", n_strips=strips, sweeps_per_launch=spl, tuning=LEXW)
    o = O.Oracle(cp, ordering=O.LEX)
    g.set_field("src", f)
    o.field("src")[...] = f
    ig, rg = g.solverPressurePoisson()
    io, ro = o.poisson()
    return g, o, (ig, rg), (io, ro)


def random_source(cp, seed=5, scale=10.0):
    rng = np.random.default_rng(seed)
    f = np.zeros((cp.ny + 2, cp.nx + 2))
    f[1:cp.ny + 1, 1:cp.nx + 1] = rng.standard_normal((cp.ny, cp.nx)) * scale
    return f


@pytest.mark.parametrize("spl", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("nx,ny,K", [(40, 24, 37), (300, 130, 25), (129, 257, 1), (129, 257, 2), (257, 64, 113),
                                     (219, 40, 29), (220, 41, 30)])
def test_capped_solve_bitexact(nx, ny, K, spl):
    cp = C.make_params("cavity", nx=nx, ny=ny, max_iters=K)
    f = random_source(cp)
    g, o, (ig, rg), (io, ro) = solve_both(cp, f, spl=spl)
    assert ig == io == K
    assert rg == ro
    assert_bits(g.field("p"), o.field("p"), f"lexw p {nx}x{ny} K={K} spl={spl}")


@pytest.mark.parametrize("strips", [2, 3])
def test_capped_solve_strips_bitexact(strips):
    cp = C.make_params("cavity", nx=200, ny=150, max_iters=41)
    f = random_source(cp, seed=9)
    g, o, (ig, rg), (io, ro) = solve_both(cp, f, strips=strips)
    assert (ig, rg) == (io, ro)
    assert_bits(g.field("p"), o.field("p"), f"lexw strips={strips}")


@pytest.mark.parametrize("spl", [2, 3, 4, 5])
def test_converging_solve_stops_at_reference_iteration(spl):
    """The reference's own 63² cavity: a realistic source (one predictor step)
    converges in a few hundred sweeps; the stop is detected up to (nx+ny)/2
    iterations late and replayed to exactly the reference's count."""
    cp = C.reference_defaults("cavity")
    g = C.CavitySolver(cp, ordering="lex", small_solve="off", sweeps_per_launch=spl, tuning=LEXW)
    o = O.Oracle(cp, ordering=O.LEX)
    g.applyBoundaryConditions()
    g.computeTentativeVelocities()
    g.buildSourceTerm()
    o.velocity_bc(False)
    o.tentative()
    o.source()
    ig, rg = g.solverPressurePoisson()
    io, ro = o.poisson()
    assert 10 < io < cp.max_iters
    assert (ig, rg) == (io, ro)
    assert_bits(g.field("p"), o.field("p"), "converged p")


@pytest.mark.parametrize("case", ["cavity_ref", "cavity_128"])
def test_whole_steps_bitexact(case):
    if case == "cavity_ref":
        cp, steps = C.reference_defaults("cavity"), 12
    else:  # BASELINE configs[0]
        cp, steps = C.make_params("cavity", re=100.0, nx=128, ny=128, dt=1e-3), 8
    g = C.CavitySolver(cp, ordering="lex", small_solve="off", tuning=LEXW)
    o = O.Oracle(cp, ordering=O.LEX)
    g.applyBoundaryConditions()
    for k in range(steps):
        assert g.step() == o.step(), k
    for name in ("u", "v", "p"):
        assert_bits(g.field(name), ofield(o, name, cp), f"{case} {name}")


def test_cavity_1024_step_bitexact_capped():
    """BASELINE configs[1] size: whole timesteps in the reference's order."""
    cp = C.make_params("cavity", re=1000.0, nx=1024, ny=1024, max_iters=150)
    g = C.CavitySolver(cp, ordering="lex", small_solve="off", tuning=LEXW)
    o = O.Oracle(cp, ordering=O.LEX)
    g.applyBoundaryConditions()
    for k in range(2):
        assert g.step() == o.step(), k
    for name in ("u", "v", "p"):
        assert_bits(g.field(name), ofield(o, name, cp), f"1024 {name}")


def test_cavity_1024_steady_launches_bitexact():
    """BASELINE configs[1] with the cap past the ramps (K = 1100 > (nx+ny)/2):
    the steady-state launches (every cell active, poisson_lexw_kernel<*, 4,
    false, *>) run and the step is bit for bit the reference loop's."""
    cp = C.make_params("cavity", re=1000.0, nx=1024, ny=1024, max_iters=1100)
    g = C.CavitySolver(cp, ordering="lex", small_solve="off", tuning=LEXW)
    o = O.Oracle(cp, ordering=O.LEX)
    g.applyBoundaryConditions()
    assert g.step() == o.step()
    assert g.timing().poisson_steady_launches > 0
    for name in ("u", "v", "p"):
        assert_bits(g.field(name), ofield(o, name, cp), f"1024 K=1100 {name}")


@pytest.mark.parametrize("spl", [0, 5])
def test_cavity_4096_step_bitexact_capped(spl):
    """The bench size: one whole timestep in the reference's order (capped)."""
    cp = C.make_params("cavity", re=1000.0, nx=4096, ny=4096, max_iters=24)
    g = C.CavitySolver(cp, ordering="lex", small_solve="off", sweeps_per_launch=spl, tuning=LEXW)
    o = O.Oracle(cp, ordering=O.LEX)
    g.applyBoundaryConditions()
    assert g.step() == o.step()
    for name in ("u", "v", "p"):
        assert_bits(g.field(name), ofield(o, name, cp), f"4096 {name}")


def test_rayleigh_benard_lex_bitexact():
    cp = C.make_params("rayleigh_benard", nx=96, ny=32, ra=2e4, max_iters=300)
    g = C.RayleighBenardSolver(cp, ordering="lex", small_solve="off")
    o = O.Oracle(cp, ordering=O.LEX)
    for k in range(6):
        assert g.step() == o.step(), k
    for name in ("u", "v", "p"):
        assert_bits(g.field(name), ofield(o, name, cp), f"RB lex {name}")


def sparse_source(cp, seed, n=6, scale=50.0):
    """A source on a few cells: near convergence the residual is concentrated
    around them, so the sampled rows (1 in 10 per band, lexw.hpp LX_SAMPLE)
    can all meet the tolerance before the reference stops - the open-iteration
    path (exact evaluation, then the continuation with every cell evaluated)."""
    rng = np.random.default_rng(seed)
    f = np.zeros((cp.ny + 2, cp.nx + 2))
    js = rng.integers(1, cp.ny + 1, n)
    is_ = rng.integers(1, cp.nx + 1, n)
    f[js, is_] = rng.standard_normal(n) * scale
    f[1:cp.ny + 1, 1:cp.nx + 1] -= f[1:cp.ny + 1, 1:cp.nx + 1].mean()
    return f


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_sampled_rows_open_iterations_exact(seed):
    """Default 3-sweep launches evaluate residuals on sampled rows. Converging
    solves from sparse sources: iteration counts, residuals and fields equal
    the reference loop's, whether the sampled stop is the reference's (exact
    check of the rebuilt field) or early (continuation). A second solve of the
    same source runs with every cell evaluated from 64 iterations before the
    first one's stop (the hint) and must agree too."""
    cp = C.make_params("cavity", nx=90, ny=70, max_iters=3000)
    cp.tol_factor = 1e-6
    f = sparse_source(cp, seed)
    g = C.CavitySolver(cp, ordering="lex", small_solve="off", tuning=LEXW)
    o = O.Oracle(cp, ordering=O.LEX)
    for rep in range(2):
        g.set_field("src", f)
        o.field("src")[...] = f
        ig, rg = g.solverPressurePoisson()
        io, ro = o.poisson()
        assert 20 < io < cp.max_iters
        assert (ig, rg) == (io, ro), rep
        assert_bits(g.field("p"), o.field("p"), f"sampled lexw seed {seed} solve {rep}")
        if rep == 0:
            assert g.timing().proof_fallbacks >= 1  # a converging sampled solve always ends open


# ---- the channel (configs[2]) in the reference's order: lexw.hpp lxo_row ----

def random_field(cp, seed, scale=1.0):
    rng = np.random.default_rng(seed)
    return rng.standard_normal((cp.ny + 2, cp.nx + 2)) * scale


def solve_channel(cp, f, p0, strips=1):
    """One solverPressurePoisson from a given source and initial pressure
    (ghosts included: the reference's first sweep reads them as stored)."""
    g = C.ChannelSolver(cp, ordering="lex", small_solve="off", n_strips=strips, tuning=LEXW)
    o = O.Oracle(cp, ordering=O.LEX)
    g.set_field("src", f)
    g.set_field("p", p0)
    o.field("src")[...] = f
    o.field("p")[...] = p0
    res_g = g.solverPressurePoisson()
    res_o = o.poisson()
    return g, o, res_g, res_o


@pytest.mark.parametrize("nx,ny,K,strips", [(93, 31, 37, 1), (300, 130, 25, 1), (129, 257, 1, 1), (129, 257, 2, 1),
                                            (257, 64, 113, 1), (200, 150, 41, 2), (200, 150, 41, 3), (224, 40, 17, 1),
                                            (225, 41, 18, 1)])
def test_channel_capped_solve_bitexact(nx, ny, K, strips):
    """Capped solves (the reference caps at 4096x512): ghosts refreshed in the
    skew, the Dirichlet outlet, arbitrary initial ghosts, odd and even widths
    (the outlet ghost in either slot), tile-edge widths, strips."""
    cp = C.make_params("channel", nx=nx, ny=ny, max_iters=K)
    f = random_field(cp, 5, 10.0)
    p0 = random_field(cp, 6)
    g, o, rg, ro = solve_channel(cp, f, p0, strips)
    assert rg[0] == ro[0] == K
    assert rg == ro
    assert_bits(g.field("p"), o.field("p"), f"channel lexw p {nx}x{ny} K={K} strips={strips}")


def test_channel_converging_solve_bitexact():
    """The reference's own channel (93x31) after one predictor step converges;
    the sampled rows leave the last iterations open and the exact check / the
    continuation must land on the reference's count."""
    cp = C.reference_defaults("channel")
    g = C.ChannelSolver(cp, ordering="lex", small_solve="off", tuning=LEXW)
    o = O.Oracle(cp, ordering=O.LEX)
    o.velocity_bc(False)
    for s in (g, ):
        s.computeTentativeVelocities()
        s.applyTentativeBoundaryConditions()
        s.buildSourceTerm()
    o.tentative()
    o.velocity_bc(True)
    o.source()
    ig, rg = g.solverPressurePoisson()
    io, ro = o.poisson()
    assert 10 < io < cp.max_iters
    assert (ig, rg) == (io, ro)
    assert_bits(g.field("p"), o.field("p"), "channel converged p")


@pytest.mark.parametrize("case", ["reference", "wide"])
def test_channel_whole_steps_bitexact(case):
    """Whole channel steps in the reference's order (the source's mean removed
    by the sequential sum), against the reference loop restated."""
    if case == "reference":
        cp, steps = C.reference_defaults("channel"), 12
    else:
        cp, steps = C.make_params("channel", re=1000.0, nx=384, ny=64, max_iters=200), 3
    g = C.ChannelSolver(cp, ordering="lex", small_solve="off", tuning=LEXW)
    o = O.Oracle(cp, ordering=O.LEX)
    o.velocity_bc(False)
    for k in range(steps):
        assert g.step() == o.step(), k
    for name in ("u", "v", "p"):
        assert_bits(g.field(name), ofield(o, name, cp), f"channel {case} {name}")


def test_channel_4096x512_step_bitexact_capped():
    """BASELINE configs[2] (channel Re=1000, 4096x512): whole timesteps in the
    reference's order, capped, bit for bit."""
    cp = C.make_params("channel", re=1000.0, nx=4096, ny=512, max_iters=30)
    g = C.ChannelSolver(cp, ordering="lex", small_solve="off", tuning=LEXW)
    o = O.Oracle(cp, ordering=O.LEX)
    o.velocity_bc(False)
    for k in range(2):
        assert g.step() == o.step(), k
    for name in ("u", "v", "p"):
        assert_bits(g.field(name), ofield(o, name, cp), f"channel 4096x512 {name}")


def test_channel_4096x512_steady_launches_bitexact():
    """BASELINE configs[2] with the cap past the ramps (K = 2320 > (nx+ny)/2):
    steady-state launches run, bit for bit the reference loop's step."""
    cp = C.make_params("channel", re=1000.0, nx=4096, ny=512, max_iters=2320)
    g = C.ChannelSolver(cp, ordering="lex", small_solve="off", tuning=LEXW)
    o = O.Oracle(cp, ordering=O.LEX)
    o.velocity_bc(False)
    assert g.step() == o.step()
    assert g.timing().poisson_steady_launches > 0
    for name in ("u", "v", "p"):
        assert_bits(g.field(name), ofield(o, name, cp), f"channel 4096x512 K=2320 {name}")


# ---- the backwards step (configs[3]) in the reference's order: lexw.hpp STEP ----

def solve_step(cp, f, p0, strips=1, solves=1):
    g = C.BackwardsStepSolver(cp, ordering="lex", small_solve="off", n_strips=strips)
    o = O.Oracle(cp, ordering=O.LEX)
    out = []
    for _ in range(solves):
        g.set_field("src", f)
        g.set_field("p", p0)
        o.field("src")[...] = f
        o.field("p")[...] = p0
        out.append((g.solverPressurePoisson(), o.poisson()))
    return g, o, out


@pytest.mark.parametrize("nx,ny,K,strips", [
    (256, 32, 37, 1),   # step_i 64, jb 17: the corner's south neighbour on an even diagonal (deferral across launches)
    (260, 34, 41, 1),   # 65, 18 (even diagonal, odd column)
    (260, 32, 29, 1),   # 65, 17 (odd diagonal)
    (256, 34, 33, 1),   # 64, 18 (odd diagonal, even column)
    (436, 32, 26, 1),   # step_i 109: the column after the step opens the second 110-column tile
    (448, 40, 1, 1), (448, 40, 2, 1), (448, 40, 113, 1),
    (300, 64, 31, 2), (300, 64, 31, 3),
])
def test_step_capped_solve_bitexact(nx, ny, K, strips):
    """Capped solves (the reference caps at every size): the solid block's
    refresh in the skew (bottom row, step column, the corner), arbitrary
    initial solids and ghosts, corner / tile-edge / parity placements, strips."""
    cp = C.make_params("backwards_step", nx=nx, ny=ny, max_iters=K)
    f = random_field(cp, 15, 10.0)
    p0 = random_field(cp, 16)
    g, o, ((rg, ro),) = solve_step(cp, f, p0, strips)
    assert rg[0] == ro[0] == K
    assert rg == ro
    assert_bits(g.field("p"), o.field("p"), f"step lexw p {nx}x{ny} K={K} strips={strips}")


@pytest.mark.parametrize("nx,ny", [(256, 32), (260, 32)])
def test_step_converging_corner_source_bitexact(nx, ny):
    """A source spiking at the corner's south neighbour (jb-1, step_i), whose
    residual is evaluated one half-sweep late (its p_N is the corner refreshed
    from the east cell's same iteration): converging solves must stop where the
    reference stops, first with sampled rows (open iterations evaluated
    exactly), then with every cell evaluated from the hint on (the deferred
    residual in the full kernels)."""
    cp = C.make_params("backwards_step", nx=nx, ny=ny, max_iters=5000)
    cp.tol_factor = 3e-3  # (converges in ~1350 sweeps; the reference's 1e-7 caps here)
    f = np.zeros((cp.ny + 2, cp.nx + 2))
    jb, si = cp.inlet_jmax + 1, cp.step_i
    f[jb - 1, si] = 40.0
    f[3, cp.nx - 5] = -25.0
    f[jb - 2, si + 3] = 7.0
    g, o, res = solve_step(cp, f, np.zeros_like(f), solves=2)
    for k, (rg, ro) in enumerate(res):
        assert 20 < ro[0] < cp.max_iters
        assert rg == ro, k
    assert_bits(g.field("p"), o.field("p"), "step converged p")


def test_step_reference_run_bitexact():
    """The reference's own step (256x32) over whole timesteps (the reference
    hits the 10000-sweep cap here from step 2: 3 steps)."""
    cp = C.reference_defaults("backwards_step")
    g = C.BackwardsStepSolver(cp, ordering="lex", small_solve="off")
    o = O.Oracle(cp, ordering=O.LEX)
    o.velocity_bc(False)
    for k in range(3):
        assert g.step() == o.step(), k
    for name in ("u", "v", "p"):
        assert_bits(g.field(name), ofield(o, name, cp), f"step reference {name}")


def test_step_8192x512_step_bitexact_capped():
    """BASELINE configs[3] (backwards step Re=400, 8192x512) on one device:
    a whole timestep in the reference's order, capped, bit for bit."""
    cp = C.make_params("backwards_step", re=400.0, nx=8192, ny=512, max_iters=24)
    g = C.BackwardsStepSolver(cp, ordering="lex", small_solve="off")
    o = O.Oracle(cp, ordering=O.LEX)
    o.velocity_bc(False)
    assert g.step() == o.step()
    for name in ("u", "v", "p"):
        assert_bits(g.field(name), ofield(o, name, cp), f"step 8192x512 {name}")


# ---- the step's column tiles left of its column (lexw.hpp left class) ----

@pytest.mark.parametrize("nx,ny,K,strips", [
    (1024, 64, 37, 1),   # step_i 256: one left tile (110-column tiles, c0 + 127 <= step_i - 1), the wall tile clipped
    (1024, 64, 1, 1), (1024, 66, 2, 1),
    (960, 34, 113, 1),   # jb 18: the edge zone spans most of the left tiles' rows
    (2000, 40, 23, 1),   # step_i 500: three left tiles
    (1100, 48, 29, 2), (1300, 40, 41, 3),  # strips (3 sweeps per launch, 112-column tiles)
])
def test_step_left_tiles_capped_bitexact(nx, ny, K, strips):
    """Capped solves with column tiles wholly left of the step's column: they
    end at the block's bottom row (refreshed as 0.0 + p_S in the skew) and the
    ghosts over the block's interior take their first-refresh values before
    the solve (step_presolid_kernel). Random initial fields: every solid and
    ghost starts off its refreshed value, so a ghost the solve did not set
    would show."""
    cp = C.make_params("backwards_step", nx=nx, ny=ny, max_iters=K)
    assert cp.step_i >= 230
    f = random_field(cp, 25, 10.0)
    p0 = random_field(cp, 26)
    g, o, ((rg, ro),) = solve_step(cp, f, p0, strips)
    assert rg[0] == ro[0] == K
    assert rg == ro
    assert_bits(g.field("p"), o.field("p"), f"step left tiles {nx}x{ny} K={K} strips={strips}")


def test_step_left_class_equals_masked_march():
    """CFD_TUNE_LEXW_LEFT 1 (default) and 0 (every march reaching the block on
    the per-cell masked path): the same whole timesteps, bit for bit, and the
    oracle's."""
    cp = C.make_params("backwards_step", re=400.0, nx=1536, ny=96, max_iters=1000)  # (> (nx+ny)/2: steady launches)
    out = []
    for left in (1, 0):
        g = C.BackwardsStepSolver(cp, ordering="lex", small_solve="off", tuning={"lexw_left": left})
        its = [g.step() for _ in range(2)]
        out.append((its, {n: g.field(n) for n in ("u", "v", "p")}))
        assert g.timing().poisson_steady_launches > 0
        g.close()
    assert out[0][0] == out[1][0]
    for n in ("u", "v", "p"):
        assert_bits(out[0][1][n], out[1][1][n], f"left class vs masked {n}")
    o = O.Oracle(cp, ordering=O.LEX)
    o.velocity_bc(False)
    assert [o.step() for _ in range(2)] == out[0][0]
    for n in ("u", "v", "p"):
        assert_bits(out[0][1][n], ofield(o, n, cp), f"left class vs oracle {n}")


def test_step_left_tiles_converging_bitexact():
    """Converging solves (early stop, replay from the initial field, the
    open-iteration continuation) with left tiles: the presolid ghosts must
    not leak into a solve that stops at iteration 0 either."""
    cp = C.make_params("backwards_step", nx=1024, ny=32, max_iters=5000)
    cp.tol_factor = 3e-3
    jb, si = cp.inlet_jmax + 1, cp.step_i
    f = np.zeros((cp.ny + 2, cp.nx + 2))
    f[jb - 1, si] = 40.0
    f[3, 100] = -25.0
    f[jb - 2, si - 50] = 7.0
    p0 = random_field(cp, 31, 1e-3)
    g, o, res = solve_step(cp, f, p0, solves=2)
    for k, (rg, ro) in enumerate(res):
        assert rg == ro, k
    assert_bits(g.field("p"), o.field("p"), "step left tiles converged p")
    # a solve with no sweep (max_iters 0; the reference's loop always sweeps
    # once otherwise): the field, ghosts included, stays as given
    cp0 = C.make_params("backwards_step", nx=1024, ny=32, max_iters=0)
    g0, o0, ((rg, ro),) = solve_step(cp0, f, p0)
    assert rg == ro and rg[0] == 0
    assert_bits(g0.field("p"), o0.field("p"), "iteration-0 stop")
