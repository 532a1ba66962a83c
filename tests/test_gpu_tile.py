"""LDS-tile red-black SOR launches (csrc/tile.hpp, poisson_tile_kernel).

A grid that fits one resident round of tiles (one 16-wave workgroup per CU,
each with its tile of p in LDS plus a 10-cell halo) runs up to 4 SOR sweeps
per launch there (3 for the step). The path must be invisible: the same
iteration counts, residuals and fields, bit for bit, as the wave-march
launches (tile_rounds 0) and as the red-black oracle — including solves that
stop inside a launch (replayed), caps around the natural stop, tile edges on
the ghost columns, the step's solid block across tiles, and plans of more
than one round.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import cfd_amd as C  # noqa: E402
import oracle as O  # noqa: E402
from cfd_amd import _lib  # noqa: E402
from test_gpu_parity import assert_bits, ofield  # noqa: E402

SOLVERS = {"cavity": C.CavitySolver, "channel": C.ChannelSolver, "backwards_step": C.BackwardsStepSolver}
FIELDS = ("p", "u", "v")
TILE_W = 108  # owned columns per tile (tile.hpp)


# the open cases run the wave march by default (faster there since the
# unchecked-group march); these tests ask for the tiles explicitly
TILES = {"tile_rounds": 1, "resident": 0}


def run(case, cp, steps, tile_rounds=None, **kw):
    tuning = {"tile_rounds": 1 if tile_rounds is None else tile_rounds, "resident": 0}
    g = SOLVERS[case](cp, ordering="rb", device=0, small_solve="off", tuning=tuning, **kw)
    if case == "cavity":
        g.applyBoundaryConditions()
    hist = [g.step() for _ in range(steps)]
    out = {n: g.field(n).copy() for n in FIELDS}
    tm = g.timing()
    g.close()
    return hist, out, tm


def params(case, nx, ny, max_iters=None, re=None):
    kw = {"nx": nx, "ny": ny}
    if max_iters is not None:
        kw["max_iters"] = max_iters
    if re is not None:
        kw["re"] = re
    return C.make_params(case, **kw)


@pytest.mark.parametrize("case,nx,ny,steps", [
    ("cavity", 300, 200, 3), ("cavity", 333, 257, 2), ("cavity", 1024, 64, 2),
    ("channel", 400, 96, 3), ("channel", 255, 130, 2),
    ("backwards_step", 400, 100, 2), ("backwards_step", 517, 131, 2),
])
def test_tile_equals_march(case, nx, ny, steps):
    cp = params(case, nx, ny, max_iters=600)
    ht, ft, tt = run(case, cp, steps)
    hm, fm, tm = run(case, cp, steps, tile_rounds=0)
    assert _lib.SOR_KERNEL[tt.sor_kernel] == "tile"
    assert _lib.SOR_KERNEL[tm.sor_kernel] == "march"
    assert ht == hm
    for n in FIELDS:
        assert_bits(ft[n], fm[n], f"{case} {nx}x{ny} {n}")
    assert tt.poisson_sweeps > 2 * tt.poisson_launches  # 3-4 sweeps per tile launch (replays: fewer)


@pytest.mark.parametrize("case", ["cavity", "channel", "backwards_step"])
@pytest.mark.parametrize("cap,tol", [(57, None), (3000, 1e-3)])
def test_tile_vs_red_black_oracle(case, cap, tol):
    """solverPressurePoisson from the same random source and initial pressure
    (ghosts included) on the tile path and in the oracle's red-black
    restatement: iteration count, residual and field bit for bit - a capped
    solve (57: inside a launch) and a converging one (a loose tolerance)."""
    cp = params(case, 240, 120, max_iters=cap)
    if tol is not None:
        cp.tol_factor = tol
    rng = np.random.default_rng(7)
    f = rng.standard_normal((cp.ny + 2, cp.nx + 2))
    p0 = rng.standard_normal((cp.ny + 2, cp.nx + 2)) * (0.0 if case == "cavity" else 1.0)
    g = SOLVERS[case](cp, ordering="rb", device=0, small_solve="off", tuning=TILES)
    o = O.Oracle(cp, ordering=O.RB)
    g.set_field("src", f)
    o.field("src")[...] = f
    g.set_field("p", p0)
    o.field("p")[...] = p0
    res_g = g.solverPressurePoisson()
    res_o = o.poisson()
    assert _lib.SOR_KERNEL[g.timing().sor_kernel] == "tile"
    assert res_g == res_o
    if tol is not None and case == "cavity":  # (the open cases' random sources need more than the cap)
        assert res_o[0] < cap
    assert_bits(g.field("p"), o.field("p"), f"{case} p after {res_o[0]} iterations")
    g.close()


@pytest.mark.parametrize("nx", [106, 107, 108, 214, 215, 216])
def test_tile_column_edges(nx):
    """Grid widths whose ghost column nx+1 lands on a tile edge (TILE_W = 108
    owned columns; nx + 2 = 108, 216, 218 ...): channel (Dirichlet outlet
    ghost, inlet ghost copy) and cavity."""
    for case in ("channel", "cavity"):
        cp = params(case, nx, 70, max_iters=400)
        ht, ft, _ = run(case, cp, 2)
        hm, fm, _ = run(case, cp, 2, tile_rounds=0)
        assert ht == hm
        for n in FIELDS:
            assert_bits(ft[n], fm[n], f"{case} nx={nx} {n}")


@pytest.mark.parametrize("spl", [1, 2, 3])
def test_tile_stop_inside_launch_and_explicit_sweeps(spl):
    """Converging solves (the reference's 63^2 cavity on the tile path): stops
    inside a launch are replayed from the launch's input; any sweep count."""
    cp = C.reference_defaults("cavity")
    g = C.CavitySolver(cp, ordering="rb", device=0, small_solve="off", sweeps_per_launch=spl, tuning=TILES)
    o = O.Oracle(cp, ordering=O.RB)
    for _ in range(3):
        assert g.step() == o.step()
    tm = g.timing()
    assert _lib.SOR_KERNEL[tm.sor_kernel] == "tile"
    assert_bits(g.field("p"), o.field("p"), f"p, {spl} sweeps per tile launch")
    g.close()


@pytest.mark.parametrize("delta", [-3, -1, 0, 1, 2, 5])
def test_tile_cap_edges(delta):
    """cap = K + delta around the natural stop K of the first solve."""
    cp = C.reference_defaults("channel")
    g = C.ChannelSolver(cp, ordering="rb", device=0, small_solve="off", tuning=TILES)
    k, _ = g.step()
    g.close()
    cp2 = C.reference_defaults("channel")
    cp2.max_iters = max(1, k + delta)
    h1, f1, t1 = run("channel", cp2, 2)
    h2, f2, _ = run("channel", cp2, 2, tile_rounds=0)
    assert _lib.SOR_KERNEL[t1.sor_kernel] == "tile"
    assert h1 == h2
    for n in FIELDS:
        assert_bits(f1[n], f2[n], f"cap {cp2.max_iters} {n}")


def test_tile_plan_of_several_rounds():
    """A grid of more tiles than CUs (tile_rounds 3) equals the march."""
    cp = params("channel", 4096, 1100, max_iters=40)
    ht, ft, tt = run("channel", cp, 1, tile_rounds=3)
    hm, fm, _ = run("channel", cp, 1, tile_rounds=0)
    assert _lib.SOR_KERNEL[tt.sor_kernel] == "tile"
    assert ht == hm
    for n in FIELDS:
        assert_bits(ft[n], fm[n], f"several rounds {n}")


@pytest.mark.parametrize("case,nx,ny,cap,tolf", [
    ("cavity", 240, 200, 3000, None), ("cavity", 333, 257, 400, None), ("channel", 300, 96, 3000, 1e-4),
    ("channel", 255, 130, 500, None), ("backwards_step", 400, 100, 3000, 1e-4), ("backwards_step", 517, 131, 300, None),
])
def test_tile_proof_mode_equals_exact(case, nx, ny, cap, tolf):
    """Proof-mode tile launches (the ring holds proof ratios; an iteration the
    proof leaves open is evaluated exactly from the launch that computed it)
    against exact residuals in every sweep: the same iteration counts,
    residuals and fields, bit for bit; converging solves take the fallback."""
    cp = params(case, nx, ny, max_iters=cap)
    if tolf is not None:
        cp.tol_factor = tolf
    hp, fp, tp = run(case, cp, 3)
    he, fe, te = run(case, cp, 3, proof_test="off")
    assert _lib.SOR_KERNEL[tp.sor_kernel] == "tile"
    assert hp == he
    for n in FIELDS:
        assert_bits(fp[n], fe[n], f"{case} {nx}x{ny} proof {n}")
    assert te.proof_fallbacks == 0
    if any(h[0] < cap for h in he):
        assert tp.proof_fallbacks >= 1  # a converging solve ends with an open iteration


def test_tile_proof_vs_oracle_converging():
    """The reference's 63^2 cavity on proof-mode tiles vs the red-black oracle."""
    cp = C.reference_defaults("cavity")
    g = C.CavitySolver(cp, ordering="rb", device=0, small_solve="off", tuning=TILES)
    o = O.Oracle(cp, ordering=O.RB)
    for _ in range(4):
        assert g.step() == o.step()
    assert g.timing().proof_fallbacks >= 1
    assert_bits(g.field("p"), o.field("p"), "p")
    g.close()
