"""The reference's order on reference-sized grids in one workgroup
(smlex.hip): bit for bit the oracle's lexicographic loop (ORC_LEX, pinned to
the reference binaries in test_oracle_golden.py) and the multi-block
reference-order march (lexw.hpp), whatever the stop: converged (replay from a
checkpoint or from the initial field) or capped (every iteration count around
the checkpoint interval M)."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import cfd_amd as C  # noqa: E402
from cfd_amd import _lib  # noqa: E402
import oracle as O  # noqa: E402


def bits_equal(a, b):
    return np.array_equal(np.asarray(a).view(np.int64), np.asarray(b).view(np.int64))


def interval(cp):  # smlex.hip smlex_interval
    m = 8
    while m < (cp.nx + cp.ny) // 6 + 2:
        m *= 2
    return m


def run_pair(cp, steps, small="auto"):
    g = C.solver_for(cp, ordering="lex", small_solve=small)
    o = O.Oracle(cp, ordering=O.LEX)
    if cp.case_id == C.params.CAVITY:
        g.applyBoundaryConditions()
    o.velocity_bc(False)
    its = []
    for k in range(steps):
        ig, rg = g.step()
        io_, ro = o.step()
        assert (ig, rg) == (io_, ro), (k, ig, io_, rg, ro)
        its.append(ig)
    nx, ny = cp.nx, cp.ny
    assert bits_equal(g.field("p"), o.field("p"))
    assert bits_equal(g.field("u"), o.field("u")[:, : nx + 1])
    assert bits_equal(g.field("v"), o.field("v")[: ny + 1, :])
    return g, its


@pytest.mark.parametrize("case,steps", [("cavity", 40), ("channel", 25), ("backwards_step", 3)])
def test_reference_defaults_run_smlex_bitexact(case, steps):
    """The reference's own runs take the one-workgroup kernel by default and
    match the oracle's reference loop bit for bit (converging solves: replay
    from a checkpoint; the step: capped solves)."""
    cp = C.reference_defaults(case)
    g, its = run_pair(cp, steps)
    assert _lib.SOR_KERNEL[g.timing().sor_kernel] == "smlex"
    assert g.timing().poisson_launches == steps  # one launch per solve


@pytest.mark.parametrize("case,nx,ny", [("cavity", 37, 21), ("cavity", 20, 45), ("channel", 50, 17),
                                        ("channel", 31, 31), ("backwards_step", 60, 20), ("backwards_step", 41, 13)])
def test_odd_grids_converging_bitexact(case, nx, ny):
    cp = C.make_params(case, nx=nx, ny=ny)
    run_pair(cp, 6)


@pytest.mark.parametrize("case", ["cavity", "channel", "backwards_step"])
def test_caps_around_checkpoints_bitexact(case):
    """Capped solves of every length around the checkpoint interval: the
    last iteration's refresh duties (ghosts / solids at the refresh after
    iteration K-1, then the final refresh), K = 1 included."""
    base = C.make_params(case, nx=40, ny=24)
    M = interval(base)
    for cap in (1, 2, 3, M - 1, M, M + 1, 2 * M + 1):
        cp = C.make_params(case, nx=40, ny=24, max_iters=cap)
        _, its = run_pair(cp, 3)
        assert all(i <= cap for i in its)


@pytest.mark.parametrize("case", ["cavity", "channel", "backwards_step"])
def test_early_convergence_replays_from_initial_field(case):
    """Solves of a sparse source (tests/test_gpu_lexw.py sparse_source) at loose
    to tight tolerances: stops before the first checkpoint (the replay restarts
    from the solve's initial field), near it and past it, each bit for bit the
    reference loop's (iteration count, residual, field)."""
    from test_gpu_lexw import sparse_source
    cp0 = C.make_params(case, nx=48, ny=30)
    M = interval(cp0)
    its = []
    for seed in (1, 2):
        for tf in (0.5, 0.2, 0.1, 0.05, 0.02, 1e-2, 1e-3, 1e-4):
            cp = C.make_params(case, nx=48, ny=30, max_iters=2000)
            cp.tol_factor = tf
            cp.abs_tol = 0.0
            # (the cavity's loop is primed with 1.0: a source of ~0.1 keeps every tolerance below it)
            f = sparse_source(cp, seed, scale=0.05 if case == "cavity" else 50.0)
            p0 = sparse_source(cp, seed + 10, scale=1e-3) if case != "cavity" else np.zeros_like(f)
            g = C.solver_for(cp, ordering="lex")
            o = O.Oracle(cp, ordering=O.LEX)
            g.set_field("src", f)
            g.set_field("p", p0)
            o.field("src")[...] = f
            o.field("p")[...] = p0
            ig, rg = g.solverPressurePoisson()
            io_, ro = o.poisson()
            assert (ig, rg) == (io_, ro), (tf, seed, ig, io_, rg, ro)
            assert bits_equal(g.field("p"), o.field("p")), (tf, seed)
            assert _lib.SOR_KERNEL[g.timing().sor_kernel] == "smlex"
            its.append(ig)
            g.close()
    assert any(1 <= i < M for i in its), its
    assert any(M < i < 2000 for i in its), its


@pytest.mark.parametrize("case,steps", [("cavity", 12), ("channel", 8), ("backwards_step", 2)])
def test_smlex_equals_multiblock_march(case, steps):
    """One workgroup vs the multi-block reference-order march (lexw.hpp) on the
    same run: the same iteration counts, residuals and fields, bit for bit."""
    cp = C.reference_defaults(case)
    a = C.solver_for(cp, ordering="lex")
    b = C.solver_for(cp, ordering="lex", small_solve="off", tuning={"resident": 0})
    if case == "cavity":
        a.applyBoundaryConditions()
        b.applyBoundaryConditions()
    for _ in range(steps):
        assert a.step() == b.step()
    assert _lib.SOR_KERNEL[a.timing().sor_kernel] == "smlex"
    assert _lib.SOR_KERNEL[b.timing().sor_kernel] == "lexw"
    for f in ("p", "u", "v"):
        assert bits_equal(a.field(f), b.field(f)), f


# grids past 4096 cells: more than 2 cells per thread and colour (MAXC 4: up to
# 8192 cells, MAXC 5: up to 10240), the cells' own values read from LDS
# (!PCREG), the source in LDS (FLDS), the cavity's multipliers rebuilt at every
# update (smlex.hip poisson_smlex_kernel)
MAXC_GRIDS = [("cavity", 70, 70, 4), ("channel", 120, 40, 4), ("backwards_step", 100, 60, 4),
              ("cavity", 96, 96, 5), ("channel", 110, 80, 5), ("backwards_step", 128, 72, 5)]


def maxc_of(nx, ny):  # smlex.hip smlex_launch
    per_colour = (nx * ny + 1) // 2
    return 2 if per_colour <= 2 * 1024 else 4 if per_colour <= 4 * 1024 else 5


@pytest.mark.parametrize("case,nx,ny,maxc", MAXC_GRIDS)
def test_maxc_variants_bitexact(case, nx, ny, maxc):
    """Whole timesteps on grids that take the MAXC 4 / 5 kernels: bit for bit
    the oracle's reference loop, one launch per solve."""
    assert maxc_of(nx, ny) == maxc
    steps = 2 if case == "backwards_step" else 4
    cp = C.make_params(case, nx=nx, ny=ny)
    g, _ = run_pair(cp, steps)
    assert _lib.SOR_KERNEL[g.timing().sor_kernel] == "smlex"
    assert g.timing().poisson_launches == steps


@pytest.mark.parametrize("case,nx,ny,maxc", MAXC_GRIDS)
def test_maxc_variants_caps_around_checkpoints_bitexact(case, nx, ny, maxc):
    """Capped solves around the checkpoint interval on the MAXC 4 / 5 grids
    (the last iteration's refresh duties and the checkpoint replay there)."""
    M = interval(C.make_params(case, nx=nx, ny=ny))
    for cap in (1, 2, M - 1, M, M + 1, 2 * M + 1):
        cp = C.make_params(case, nx=nx, ny=ny, max_iters=cap)
        g, its = run_pair(cp, 2)
        assert all(i <= cap for i in its)
        assert _lib.SOR_KERNEL[g.timing().sor_kernel] == "smlex"


@pytest.mark.parametrize("nx,ny,kernel", [(110, 88, "smlex"), (140, 69, "resident")])
def test_lds_limit_boundary(nx, ny, kernel):
    """smlex_fits past 4096 cells: p and the source both in LDS, 2 (nx+2)(ny+2)
    <= SMLEX_CELLS = 20160. (nx+2)(ny+2) = 10080 fits, 10082 does not; the
    grid that does not fit runs the resident launch (the cavity and the
    channel; the step the multi-block march), bit for bit the same."""
    assert (nx + 2) * (ny + 2) == (10080 if kernel == "smlex" else 10082)
    cp = C.make_params("cavity", nx=nx, ny=ny)
    g, _ = run_pair(cp, 2)
    assert _lib.SOR_KERNEL[g.timing().sor_kernel] == kernel


def test_large_grid_keeps_multiblock_march():
    """Past the LDS (grids over 4096 cells: p and the source in LDS,
    2 (nx+2)(ny+2) <= SMLEX_CELLS = 20160; up to 4096 cells: (nx+2)(ny+2) <=
    20160) the reference order runs the resident launch (the cavity, where one
    tile per CU covers the grid) or the multi-block march."""
    g = C.solver_for(C.make_params("cavity", nx=128, ny=128), ordering="lex")
    g.applyBoundaryConditions()
    g.step()
    assert _lib.SOR_KERNEL[g.timing().sor_kernel] == "resident"
    g = C.solver_for(C.make_params("cavity", nx=128, ny=128), ordering="lex", tuning={"resident": 0})
    g.applyBoundaryConditions()
    g.step()
    assert _lib.SOR_KERNEL[g.timing().sor_kernel] == "lexw"
