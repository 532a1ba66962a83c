"""Register-resident red-black SOR solve (csrc/resident.hpp, poisson_resident_kernel).

One persistent launch runs the whole capped cavity solve with every tile of p
(and the source) in registers, exchanging 8-cell edge bands through global
memory every 4 sweeps and proving "the reference goes on" per iteration
(cavity-01.cpp:633-678). The path must be invisible: the same iteration counts,
residuals and fields, bit for bit, as the LDS-tile / march launches and as the
red-black oracle - including converging solves (an iteration the proof leaves
open: the launch exits, the host replays to that group's first iteration and
finishes with exact residuals), caps around the natural stop, tile edges on the
ghost columns and rows, and the BASELINE configs[1] size.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import cfd_amd as C  # noqa: E402
import oracle as O  # noqa: E402
from cfd_amd import _lib  # noqa: E402
from test_gpu_parity import assert_bits, ofield  # noqa: E402

FIELDS = ("p", "u", "v")
RES_TW = {"rb": 112, "lex cavity": 96, "lex channel": 104}  # owned columns per tile (resident.hpp res_tw)


def run(cp, steps, resident=True, **kw):
    tuning = {"resident": 1 if resident else 0, "tile_rounds": 1}
    g = C.CavitySolver(cp, ordering="rb", device=0, small_solve="off", tuning=tuning, **kw)
    g.applyBoundaryConditions()
    hist = [g.step() for _ in range(steps)]
    out = {n: g.field(n).copy() for n in FIELDS}
    tm = g.timing()
    g.close()
    return hist, out, tm


def params(nx, ny, max_iters=None, tol=None):
    kw = {"nx": nx, "ny": ny}
    if max_iters is not None:
        kw["max_iters"] = max_iters
    cp = C.make_params("cavity", **kw)
    if tol is not None:
        cp.tol_factor = tol
    return cp


@pytest.mark.parametrize("nx,ny,steps,cap", [
    (300, 200, 3, 600), (333, 257, 2, 401), (1024, 64, 2, 600), (113, 130, 3, 500), (110, 110, 2, 300),
    (222, 96, 2, 403), (223, 40, 2, 300), (500, 300, 2, 1001),
])
def test_resident_equals_tiles(nx, ny, steps, cap):
    """Capped solves (odd caps: a short last group) on grids whose ghost
    column / row lands on or next to a tile edge (nx + 2 = 112, 224, 225...)."""
    cp = params(nx, ny, max_iters=cap)
    hr, fr, tr = run(cp, steps)
    ht, ft, tt = run(cp, steps, resident=False)
    assert _lib.SOR_KERNEL[tr.sor_kernel] == "resident"
    assert _lib.SOR_KERNEL[tt.sor_kernel] in ("tile", "march")
    assert hr == ht
    for n in FIELDS:
        assert_bits(fr[n], ft[n], f"{nx}x{ny} {n}")
    if tr.proof_fallbacks == 0:  # (late iterations of a capped solve may sit inside the proof's margin)
        assert tr.poisson_launches == steps  # the whole solve in one launch


@pytest.mark.parametrize("cap,tol", [(57, None), (3000, 1e-3), (3000, 1e-2)])
def test_resident_vs_red_black_oracle(cap, tol):
    """solverPressurePoisson from one random source on the resident path and in
    the oracle's red-black restatement: iteration count, residual and field
    bit for bit - capped (57: inside a group) and converging (loose
    tolerances: the proof leaves an iteration open, exact launches finish)."""
    cp = params(240, 120, max_iters=cap, tol=tol)
    rng = np.random.default_rng(7)
    f = rng.standard_normal((cp.ny + 2, cp.nx + 2))
    g = C.CavitySolver(cp, ordering="rb", device=0, small_solve="off", tuning={"resident": 1})
    o = O.Oracle(cp, ordering=O.RB)
    g.set_field("src", f)
    o.field("src")[...] = f
    res_g = g.solverPressurePoisson()
    res_o = o.poisson()
    tm = g.timing()
    assert _lib.SOR_KERNEL[tm.sor_kernel] == "resident"
    assert res_g == res_o
    if tol is not None:
        assert res_o[0] < cap
        assert tm.proof_fallbacks >= 1
    assert_bits(g.field("p"), o.field("p"), f"p after {res_o[0]} iterations")
    g.close()


def test_resident_reference_run_vs_oracle():
    """The reference's own 63^2 cavity (every solve converges) on the resident
    path: each solve ends in the fallback; whole steps bit for bit."""
    cp = C.reference_defaults("cavity")
    g = C.CavitySolver(cp, ordering="rb", device=0, small_solve="off", tuning={"resident": 1})
    o = O.Oracle(cp, ordering=O.RB)
    for _ in range(4):
        assert g.step() == o.step()
    tm = g.timing()
    assert _lib.SOR_KERNEL[tm.sor_kernel] == "resident"
    assert tm.proof_fallbacks >= 4
    assert_bits(g.field("p"), o.field("p"), "p")
    assert_bits(g.field("u"), o.field("u")[:, : cp.nx + 1], "u")
    g.close()


@pytest.mark.parametrize("delta", [-5, -4, -3, -1, 0, 1, 2, 5])
def test_resident_cap_edges(delta):
    """cap = K + delta around the natural stop K of the first solve (the
    stop's group, the groups before it, the cap inside the checked lag)."""
    cp = params(200, 150)
    g = C.CavitySolver(cp, ordering="rb", device=0, small_solve="off", tuning={"resident": 0})
    g.applyBoundaryConditions()
    k, _ = g.step()
    g.close()
    cp2 = params(200, 150, max_iters=max(1, k + delta))
    h1, f1, t1 = run(cp2, 2)
    h2, f2, _ = run(cp2, 2, resident=False)
    assert _lib.SOR_KERNEL[t1.sor_kernel] == "resident"
    assert h1 == h2
    for n in FIELDS:
        assert_bits(f1[n], f2[n], f"cap {cp2.max_iters} {n}")


def test_resident_baseline_1024_capped():
    """BASELINE configs[1] (cavity Re=1000, 1024^2): two whole capped steps
    (10000 sweeps each) equal the LDS-tile launches bit for bit; the second
    step's solve is one launch with no fallback (the first step's first
    iteration is left open by the proof on every path: DESIGN.md §2)."""
    cp = C.make_params("cavity", nx=1024, ny=1024)
    g = C.CavitySolver(cp, ordering="rb", device=0, small_solve="off", tuning={"resident": 1})
    g.applyBoundaryConditions()
    hr = [g.step()]
    g.reset_timing()
    hr.append(g.step())
    tr = g.timing()
    fr = {n: g.field(n).copy() for n in FIELDS}
    g.close()
    ht, ft, _ = run(cp, 2, resident=False)
    assert _lib.SOR_KERNEL[tr.sor_kernel] == "resident"
    assert hr == ht and hr[1][0] == cp.max_iters
    for n in FIELDS:
        assert_bits(fr[n], ft[n], f"1024^2 {n}")
    assert tr.poisson_launches == 1 and tr.proof_fallbacks == 0


def test_resident_not_planned_beyond_one_tile_per_cu():
    """A grid of more tiles than CUs keeps the per-launch kernels."""
    cp = params(2048, 2048, max_iters=8)
    _, _, tm = run(cp, 1)
    assert _lib.SOR_KERNEL[tm.sor_kernel] != "resident"


# ---- the reference's own order (resident.hip LEX): the one-device default ----

def run_lex(cp, steps, resident=True, **kw):
    """steps whole steps; the timing covers steps 2.. (the first solve from
    rest has exceedances only at the lid's corners for its first iterations,
    cells the sampler skips: it may take the exact path)."""
    g = C.CavitySolver(cp, ordering="lex", device=0, small_solve="off", tuning={"resident": 1 if resident else 0}, **kw)
    g.applyBoundaryConditions()
    hist = [g.step()]
    g.reset_timing()
    hist += [g.step() for _ in range(steps - 1)]
    out = {n: g.field(n).copy() for n in FIELDS}
    tm = g.timing()
    g.close()
    return hist, out, tm


@pytest.mark.parametrize("nx,ny,steps,cap", [
    (300, 200, 3, 600), (333, 257, 3, 401), (1024, 64, 3, 600), (113, 130, 3, 500), (110, 110, 3, 300),
    (222, 96, 3, 403), (500, 300, 3, 1001), (100, 400, 3, 700),
    (94, 80, 3, 500), (190, 90, 3, 403), (191, 60, 3, 300), (1024, 1100, 2, 300),
])
def test_resident_lex_equals_lexw(nx, ny, steps, cap):
    """Capped solves in the reference's order: the resident launch (ramps
    masked, residuals sampled; 8-sweep groups of 96-column tiles: nx + 2 =
    96, 192, 193 on tile edges; 1024x1100: 80-row regions of 10-row waves)
    against the multi-launch march lexw.hpp, which is bit-exact vs the
    reference loop (tests/test_gpu_lexw.py)."""
    cp = params(nx, ny, max_iters=cap)
    hr, fr, tr = run_lex(cp, steps)
    hw, fw, tw = run_lex(cp, steps, resident=False)
    assert _lib.SOR_KERNEL[tr.sor_kernel] == "resident"
    assert _lib.SOR_KERNEL[tw.sor_kernel] == "lexw"
    assert hr == hw
    for n in FIELDS:
        assert_bits(fr[n], fw[n], f"lex {nx}x{ny} {n}")
    assert tr.proof_fallbacks == 0 and tr.poisson_launches == steps - 1


@pytest.mark.parametrize("cap,tol", [(57, None), (5000, 1e-3), (5000, 1e-2)])
def test_resident_lex_vs_reference_order_oracle(cap, tol):
    """solverPressurePoisson from one random source in the reference's order
    (ORC_LEX = the reference loop, pinned against the reference binary):
    capped, and converging (the stop iteration has no sampled exceedance: the
    exact path takes over) - iteration count, residual and field bit for bit."""
    cp = params(160, 100, max_iters=cap, tol=tol)
    rng = np.random.default_rng(11)
    f = rng.standard_normal((cp.ny + 2, cp.nx + 2))
    g = C.CavitySolver(cp, ordering="lex", device=0, small_solve="off", tuning={"resident": 1})
    o = O.Oracle(cp, ordering=O.LEX)
    g.set_field("src", f)
    o.field("src")[...] = f
    res_g = g.solverPressurePoisson()
    res_o = o.poisson()
    tm = g.timing()
    assert _lib.SOR_KERNEL[tm.sor_kernel] == "resident"
    assert res_g == res_o
    if tol is not None:
        assert res_o[0] < cap and tm.proof_fallbacks >= 1
    assert_bits(g.field("p"), o.field("p"), f"lex p after {res_o[0]} iterations")
    g.close()


def test_resident_lex_reference_run_vs_oracle():
    """The reference's own 63^2 run (every solve converges) forced onto the
    resident path (small_solve off): each solve falls back to the exact
    path; whole steps bit for bit with the reference loop."""
    cp = C.reference_defaults("cavity")
    g = C.CavitySolver(cp, ordering="lex", device=0, small_solve="off", tuning={"resident": 1})
    o = O.Oracle(cp, ordering=O.LEX)
    for _ in range(3):
        assert g.step() == o.step()
    assert_bits(g.field("p"), o.field("p"), "p")
    assert_bits(g.field("u"), o.field("u")[:, : cp.nx + 1], "u")
    g.close()


def test_resident_lex_baseline_1024_capped():
    """BASELINE configs[1] (1024^2, cap 10000) in the reference's order: one
    whole step per launch equals lexw.hpp bit for bit."""
    cp = C.make_params("cavity", nx=1024, ny=1024)
    hr, fr, tr = run_lex(cp, 2)
    hw, fw, _ = run_lex(cp, 2, resident=False)
    assert _lib.SOR_KERNEL[tr.sor_kernel] == "resident"
    assert hr == hw and hr[1][0] == cp.max_iters
    for n in FIELDS:
        assert_bits(fr[n], fw[n], f"lex 1024^2 {n}")
    assert tr.poisson_launches == 1 and tr.proof_fallbacks == 0


# ---- the channel (configs[2]) in the reference's order: resident.hip res_half_open ----

RES = {"resident": 1}


def channel_solve(cp, f, p0, resident=True):
    g = C.ChannelSolver(cp, ordering="lex", small_solve="off", tuning={"resident": 1 if resident else 0})
    g.set_field("src", f)
    g.set_field("p", p0)
    r = g.solverPressurePoisson()
    out = g.field("p").copy()
    tm = g.timing()
    g.close()
    return r, out, tm


@pytest.mark.parametrize("nx,ny,K", [(93, 31, 37), (300, 130, 25), (257, 64, 113), (224, 40, 17), (225, 41, 18),
                                     (110, 120, 60), (222, 300, 41), (500, 200, 301), (1000, 60, 200),
                                     (102, 50, 33), (206, 70, 41), (207, 45, 19), (208, 66, 23)])
def test_resident_channel_lex_vs_reference_order_oracle(nx, ny, K):
    """Capped channel solves from an arbitrary pressure (ghosts and corners
    included: the first sweep reads the ghosts as stored; the corners are never
    written) on the resident launch: the ghost refreshes in the skew (left /
    bottom two half-sweeps late), the outlet's zero, outlet ghost in either
    slot and on tile edges (nx + 2 = 224 / 225 / 226 / 112 ...), several row tiles."""
    cp = C.make_params("channel", nx=nx, ny=ny, max_iters=K)
    rng = np.random.default_rng(nx + ny)
    f = rng.standard_normal((ny + 2, nx + 2)) * 10.0
    p0 = rng.standard_normal((ny + 2, nx + 2))
    r, p, tm = channel_solve(cp, f, p0)
    o = O.Oracle(cp, ordering=O.LEX)
    o.field("src")[...] = f
    o.field("p")[...] = p0
    ro = o.poisson()
    assert _lib.SOR_KERNEL[tm.sor_kernel] == "resident"
    assert r == ro and ro[0] == K
    assert_bits(p, o.field("p"), f"channel resident {nx}x{ny} K={K}")
    assert tm.proof_fallbacks == 0 and tm.poisson_launches == 1


def test_resident_channel_lex_equals_lexw_converging():
    """Converging channel solves (a 240x80 channel's first steps: each solve
    stops before the cap): the resident launch leaves the stop open, the exact
    path (lexw.hpp) takes over from the untouched input - the same counts,
    residuals and fields as lexw alone."""
    cp = C.make_params("channel", nx=240, ny=80, max_iters=20000)
    cp.tol_factor = 1e-3  # (stops at 7915, 11347, 2117: the reference loop restated)
    out = []
    for r in (1, 0):
        g = C.ChannelSolver(cp, ordering="lex", small_solve="off", tuning={"resident": r})
        hist = [g.step() for _ in range(3)]
        out.append((hist, g.field("p").copy(), g.field("u").copy(), g.timing()))
        g.close()
    (h1, p1, u1, t1), (h2, p2, u2, t2) = out
    assert _lib.SOR_KERNEL[t1.sor_kernel] == "resident" and _lib.SOR_KERNEL[t2.sor_kernel] == "lexw"
    assert h1 == h2 and all(k < cp.max_iters for k, _ in h1)
    assert t1.proof_fallbacks >= 1
    assert_bits(p1, p2, "channel converging p")
    assert_bits(u1, u2, "channel converging u")


@pytest.mark.parametrize("case", ["reference", "wide"])
def test_resident_channel_whole_steps_vs_oracle(case):
    """Whole channel steps (reference 93x31: every solve converges; 384x64
    capped) with the resident launch, against the reference loop restated."""
    if case == "reference":
        cp, steps = C.reference_defaults("channel"), 6
    else:
        cp, steps = C.make_params("channel", re=1000.0, nx=384, ny=64, max_iters=200), 3
    g = C.ChannelSolver(cp, ordering="lex", small_solve="off", tuning=RES)
    o = O.Oracle(cp, ordering=O.LEX)
    o.velocity_bc(False)
    for k in range(steps):
        assert g.step() == o.step(), k
    assert _lib.SOR_KERNEL[g.timing().sor_kernel] == "resident"
    for name in ("u", "v", "p"):
        assert_bits(g.field(name), ofield(o, name, cp), f"channel resident {case} {name}")
    g.close()


@pytest.mark.parametrize("K", [30, 2320])
def test_resident_channel_4096x512_vs_oracle(K):
    """BASELINE configs[2] (channel Re=1000, 4096x512: 37 x 6 tiles of 14-row
    waves): a whole step, capped inside the ramps (30) and past them (2320),
    one launch, bit for bit the reference loop's step."""
    cp = C.make_params("channel", re=1000.0, nx=4096, ny=512, max_iters=K)
    g = C.ChannelSolver(cp, ordering="lex", small_solve="off", tuning=RES)
    o = O.Oracle(cp, ordering=O.LEX)
    o.velocity_bc(False)
    assert g.step() == o.step()
    tm = g.timing()
    assert _lib.SOR_KERNEL[tm.sor_kernel] == "resident"
    if tm.proof_fallbacks == 0:  # (a first step from rest may have no sampled exceedance early on)
        assert tm.poisson_launches == 1
    for name in ("u", "v", "p"):
        assert_bits(g.field(name), ofield(o, name, cp), f"channel 4096x512 K={K} {name}")
    g.close()


# ---- the channel (configs[2]) in red-black order: ghosts as cells of their colour ----

def channel_rb(cp, f, p0, resident=True):
    g = C.ChannelSolver(cp, ordering="rb", small_solve="off", tuning={"resident": 1 if resident else 0})
    g.set_field("src", f)
    g.set_field("p", p0)
    r = g.solverPressurePoisson()
    out = g.field("p").copy()
    tm = g.timing()
    g.close()
    return r, out, tm


@pytest.mark.parametrize("nx,ny,K", [(240, 120, 57), (93, 31, 37), (300, 130, 25), (224, 40, 17), (225, 41, 18),
                                     (110, 120, 60), (222, 300, 41), (500, 200, 301), (1000, 60, 203), (240, 120, 1),
                                     (240, 120, 4), (240, 120, 5)])
def test_resident_channel_rb_vs_red_black_oracle(nx, ny, K):
    """Capped channel solves from an arbitrary pressure (ghosts and corners
    included) on the resident launch: the red ghosts keep their stored values
    in the first half-sweep and take the last refresh after the launch, the
    outlet's zero, ghosts on tile edges, short last groups (K mod 4) - against
    the oracle's red-black restatement, bit for bit."""
    cp = C.make_params("channel", nx=nx, ny=ny, max_iters=K)
    rng = np.random.default_rng(nx * 7 + ny)
    f = rng.standard_normal((ny + 2, nx + 2)) * 10.0
    p0 = rng.standard_normal((ny + 2, nx + 2))
    r, p, tm = channel_rb(cp, f, p0)
    o = O.Oracle(cp, ordering=O.RB)
    o.field("src")[...] = f
    o.field("p")[...] = p0
    ro = o.poisson()
    assert _lib.SOR_KERNEL[tm.sor_kernel] == "resident"
    assert r == ro and ro[0] == K
    assert_bits(p, o.field("p"), f"channel rb resident {nx}x{ny} K={K}")
    if tm.proof_fallbacks == 0:
        assert tm.poisson_launches == 1


def test_resident_channel_rb_converging_equals_march():
    """Converging channel solves (240x80, loose tolerance, three steps): the
    proof leaves the stop's group open, the replay and the exact launches
    finish - the same counts, residuals and fields as the march alone."""
    cp = C.make_params("channel", nx=240, ny=80, max_iters=20000)
    cp.tol_factor = 1e-3
    out = []
    for r in (1, 0):
        g = C.ChannelSolver(cp, ordering="rb", small_solve="off", tuning={"resident": r})
        hist = [g.step() for _ in range(3)]
        out.append((hist, g.field("p").copy(), g.field("u").copy(), g.timing()))
        g.close()
    (h1, p1, u1, t1), (h2, p2, u2, t2) = out
    assert _lib.SOR_KERNEL[t1.sor_kernel] == "resident" and _lib.SOR_KERNEL[t2.sor_kernel] != "resident"
    assert h1 == h2 and all(k < cp.max_iters for k, _ in h1)
    assert t1.proof_fallbacks >= 1
    assert_bits(p1, p2, "channel rb converging p")
    assert_bits(u1, u2, "channel rb converging u")


@pytest.mark.parametrize("case", ["reference", "wide"])
def test_resident_channel_rb_whole_steps_equal_march(case):
    """Whole red-black channel steps (reference 93x31: every solve converges;
    384x64 capped) on the resident launch and on the march launches: counts,
    residuals and fields bit for bit. (Against the oracle the red-black
    channel step differs in the source's mean removal - a tree sum here, the
    sequential sum only in the reference's order: test_gpu_parity.py - so the
    march, itself pinned to the oracle solve by solve, is the reference.)"""
    if case == "reference":
        cp, steps = C.reference_defaults("channel"), 6
    else:
        cp, steps = C.make_params("channel", re=1000.0, nx=384, ny=64, max_iters=200), 3
    out = []
    for r in (1, 0):
        g = C.ChannelSolver(cp, ordering="rb", small_solve="off", tuning={"resident": r})
        hist = [g.step() for _ in range(steps)]
        out.append((hist, {n: g.field(n).copy() for n in ("u", "v", "p")}, g.timing()))
        g.close()
    (h1, f1, t1), (h2, f2, t2) = out
    assert _lib.SOR_KERNEL[t1.sor_kernel] == "resident" and _lib.SOR_KERNEL[t2.sor_kernel] != "resident"
    assert h1 == h2
    for name in ("u", "v", "p"):
        assert_bits(f1[name], f2[name], f"channel rb resident {case} {name}")


def test_resident_channel_rb_4096x512_equals_march():
    """BASELINE configs[2] (channel Re=1000, 4096x512, cap 10000): two whole
    red-black steps on the resident launch (14-row waves) equal the march
    launches bit for bit; the second solve is one launch."""
    cp = C.make_params("channel", re=1000.0, nx=4096, ny=512)
    out = []
    for r in (1, 0):
        g = C.ChannelSolver(cp, ordering="rb", small_solve="off", tuning={"resident": r})
        hist = [g.step()]
        g.reset_timing()
        hist.append(g.step())
        out.append((hist, {n: g.field(n).copy() for n in FIELDS}, g.timing()))
        g.close()
    (h1, f1, t1), (h2, f2, _) = out
    assert _lib.SOR_KERNEL[t1.sor_kernel] == "resident"
    assert h1 == h2 and h1[1][0] == cp.max_iters
    for n in FIELDS:
        assert_bits(f1[n], f2[n], f"channel rb 4096x512 {n}")
    assert t1.poisson_launches == 1 and t1.proof_fallbacks == 0


@pytest.mark.parametrize("order", ["rb", "lex"])
@pytest.mark.parametrize("case", ["cavity", "channel"])
def test_resident_check_every_equals_per_launch_paths(case, order):
    """check_every = 3 through converging solves: red-black tests multiples
    of 3 only (the resident launch's proofs of the tested iterations, its
    fallback), the reference order every iteration as lexw.hpp and smlex.hip
    do - the same counts, residuals and fields as the per-launch kernels."""
    cp = C.make_params(case, nx=240, ny=80, max_iters=20000)
    cp.tol_factor = 1e-3
    out = []
    for r in (1, 0):
        g = C.solver_for(cp, ordering=order, small_solve="off", check_every=3, tuning={"resident": r})
        if case == "cavity":
            g.applyBoundaryConditions()
        hist = [g.step() for _ in range(3)]
        out.append((hist, g.field("p").copy(), g.timing()))
        g.close()
    (h1, p1, t1), (h2, p2, t2) = out
    assert _lib.SOR_KERNEL[t1.sor_kernel] == "resident" and _lib.SOR_KERNEL[t2.sor_kernel] != "resident"
    assert h1 == h2
    if order == "rb":
        assert all(k % 3 == 0 or k == cp.max_iters for k, _ in h1)
    assert_bits(p1, p2, f"{case} {order} check_every 3 p")


# ---- a solve from rest returns to the resident launch (round 6) ----

@pytest.mark.parametrize("order", ["rb", "lex"])
def test_resident_step_from_rest_returns_to_resident(order):
    """BASELINE configs[1] (1024^2, cap 10000) from rest: the first solve's
    first iterations have residuals only at the lid's corners (no proof, no
    sampled row), so the resident launch leaves an iteration open; an exact
    window of launches settles that stretch and the resident kernel takes the
    rest of the solve again (Solver::solve_resident_segments) - a handful of
    launches, not the ~2500 exact ones of round 5 - and both steps stay bit
    for bit the per-launch path's (LDS tiles / lexw). The first step's time
    is printed beside the second's."""
    cp = C.make_params("cavity", nx=1024, ny=1024)
    g = C.CavitySolver(cp, ordering=order, device=0, small_solve="off", tuning={"resident": 1})
    g.applyBoundaryConditions()
    hist = [g.step()]
    t1 = g.timing()
    g.reset_timing()
    hist.append(g.step())
    t2 = g.timing()
    fr = {n: g.field(n).copy() for n in FIELDS}
    g.close()
    tuning = {"resident": 0, "tile_rounds": 1}
    w = C.CavitySolver(cp, ordering=order, device=0, small_solve="off", tuning=tuning)
    w.applyBoundaryConditions()
    hw = [w.step() for _ in range(2)]
    fw = {n: w.field(n).copy() for n in FIELDS}
    w.close()
    assert hist == hw and hist[0][0] == cp.max_iters
    for n in FIELDS:
        assert_bits(fr[n], fw[n], f"{order} from rest {n}")
    assert _lib.SOR_KERNEL[t1.sor_kernel] == "resident"
    assert t1.proof_fallbacks >= 1  # (the open iteration at the start)
    # (red-black: one exact window of 32 launches; the reference order's window
    # pays the skew's ramps, ~(nx + ny) / 8 launches)
    assert t1.poisson_launches <= (80 if order == "rb" else 400), t1.poisson_launches
    assert t2.poisson_launches == 1
    print(f"\n{order}: step 1 {t1.poisson_ms:.2f} ms in {t1.poisson_launches} launches, step 2 {t2.poisson_ms:.2f} ms"
          f" ({t1.poisson_ms / t2.poisson_ms:.2f}x)")


def test_resident_timeout_fallback_plan_is_co_resident():
    """The plan only takes the persistent launch when the occupancy query
    admits every tile at once (res_coresident_tiles): no resident solve of
    the suite timed out."""
    cp = C.make_params("cavity", nx=1024, ny=1024, max_iters=40)
    g = C.CavitySolver(cp, ordering="lex", device=0, small_solve="off", tuning={"resident": 1})
    g.applyBoundaryConditions()
    g.step()
    tm = g.timing()
    g.close()
    assert _lib.SOR_KERNEL[tm.sor_kernel] == "resident" and tm.resident_timeouts == 0
