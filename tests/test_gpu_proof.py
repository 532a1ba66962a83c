"""Proof-mode convergence test of the red-black cavity launches
(kernels.hpp `proof_ratio`).

The reference sweeps while max|r| > tol (cavity-01.cpp:633). A proof-mode
launch does not evaluate the residual: it proves "some cell has |r| > tol"
from the size of its black updates (r = K (p' - p) + rounding terms it
bounds), and an iteration it cannot settle that way is evaluated exactly (the
solve restarts, with the exact residual kernel, at the launch that computed
it). The test must be invisible: the same iteration counts, the same reported
residuals and the same fields, bit for bit, as exact residuals throughout
(proof_test="off") and as the red-black oracle.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import cfd_amd as C  # noqa: E402
import oracle as O  # noqa: E402
from test_gpu_parity import assert_bits  # noqa: E402

FIELDS = ("p", "u", "v")
MARCH = {"tile_rounds": 0, "resident": 0}  # the wave-march launches (proof mode runs there), not the LDS tiles


def run(monkeypatch, cp, steps, proof, ns=3, last_timing=False, **kw):
    """proof: the proof-mode test with `ns` sweeps per launch (3, or 4: no
    residual stage, so four sweeps fit the 8-row halos); else exact residuals.
    Always the multi-launch solve (small_solve off), at any size.
    last_timing: timing of the last step only."""
    g = C.CavitySolver(cp, ordering="rb", device=0, small_solve="off", tuning=MARCH, proof_test="on" if proof else "off",
                       sweeps_per_launch=ns if proof else 0, **kw)
    hist = []
    for s in range(steps):
        if last_timing and s == steps - 1:
            g.reset_timing()
        hist.append(g.step())
    out = {n: g.field(n).copy() for n in FIELDS}
    tm = g.timing()
    g.close()
    return hist, out, tm


def same(a, b, what):
    (h0, f0, _), (h1, f1, _) = a, b
    assert h1 == h0, what
    for n in FIELDS:
        assert_bits(f1[n], f0[n], f"{what} {n}")


@pytest.mark.parametrize("ns", [3, 4])
@pytest.mark.parametrize("nx,ny", [(240, 200), (357, 290)])
def test_converging_solves_fall_back_and_match_oracle(monkeypatch, nx, ny, ns):
    """Solves that converge: the proof settles the early iterations, the last
    ones near the tolerance are evaluated exactly (fallback), and the stop
    lands on the reference's iteration."""
    cp = C.make_params("cavity", nx=nx, ny=ny)
    ex = run(monkeypatch, cp, 3, False)
    pr = run(monkeypatch, cp, 3, True, ns)
    same(ex, pr, f"proof ({ns} sweeps) vs exact {nx}x{ny}")
    assert ex[2].proof_fallbacks == 0
    converged = [k for k, _ in ex[0] if k < cp.max_iters]
    assert converged, "fixture meant to converge"
    assert pr[2].proof_fallbacks >= len(converged)
    o = O.Oracle(cp, ordering=O.RB)
    ho = [o.step() for _ in range(3)]
    assert ho == ex[0]
    assert_bits(pr[1]["p"], o.field("p"), "p vs oracle")


@pytest.mark.parametrize("ns", [3, 4])
@pytest.mark.parametrize("cap", [30, 31, 32, 33, 34, 35, 100])
def test_capped_solves_never_fall_back(monkeypatch, cap, ns):
    """Capped solves far from convergence (1024^2, BASELINE configs[1]): every
    iteration proven, shorter last launches (n = 1, 2) test the proof ratios
    of the launch before, the host tests the last ones; the reported residual
    is recomputed from the final field and equals the exact launches' one.
    (The first timestep's source lives in the two lid corners only, so its
    first sweep moves no cell that can prove: one fallback there, by design;
    the second step must need none.)"""
    cp = C.make_params("cavity", nx=1024, ny=1024, max_iters=cap)
    ex = run(monkeypatch, cp, 2, False)
    pr = run(monkeypatch, cp, 2, True, ns, last_timing=True)
    same(ex, pr, f"cap {cap}, {ns} sweeps")
    assert pr[2].proof_fallbacks == 0
    assert all(k == cap for k, _ in pr[0])


@pytest.mark.parametrize("ns", [3, 4])
@pytest.mark.parametrize("check_every", [1, 8])
def test_strips_and_check_every(monkeypatch, check_every, ns):
    cp = C.make_params("cavity", nx=300, ny=260)
    ex = run(monkeypatch, cp, 2, False, check_every=check_every)
    pr = run(monkeypatch, cp, 2, True, ns, check_every=check_every, n_strips=3)
    same(ex, pr, f"3 strips, check_every {check_every}")


@pytest.mark.parametrize("ns", [3, 4])
@pytest.mark.parametrize("delta", [-4, -1, 0, 1, 2, 5])
def test_cap_around_the_natural_stop(monkeypatch, delta, ns):
    """Caps just below / at / above the converged iteration: the fallback and
    the cap meet in every order."""
    cp = C.make_params("cavity", nx=240, ny=200)
    K = run(monkeypatch, cp, 1, False)[0][0][0]
    assert K < cp.max_iters
    cp2 = C.make_params("cavity", nx=240, ny=200, max_iters=K + delta)
    same(run(monkeypatch, cp2, 1, False), run(monkeypatch, cp2, 1, True, ns), f"cap K{delta:+d}")


@pytest.mark.parametrize("ns", [3, 4])
def test_full_size_step_proven(monkeypatch, ns):
    """The bench's grid (4096^2), 61 capped sweeps: after the first step (see
    above) the proof settles every iteration, and the fields equal the exact
    launches'."""
    cp = C.make_params("cavity", nx=4096, ny=4096, max_iters=61)
    ex = run(monkeypatch, cp, 2, False)
    pr = run(monkeypatch, cp, 2, True, ns, last_timing=True)
    same(ex, pr, f"4096^2, {ns} sweeps")
    assert pr[2].proof_fallbacks == 0


def solve_source(cp, f, proof, chunk=0):
    """solverPressurePoisson on a given source (cavity: from a zero field)."""
    g = C.CavitySolver(cp, ordering="rb", device=0, small_solve="off", tuning=MARCH, proof_test="on" if proof else "off",
                       sweeps_per_launch=4 if proof else 0, chunk=chunk)
    g.set_field("src", f)
    it, res = g.solverPressurePoisson()
    p = g.field("p").copy()
    g.close()
    return (it, res), p


def test_stop_in_first_proof_launch_after_fallback():
    """The first proof-mode launch after a fallback follows exact 3-sweep
    launches and runs 4 sweeps: before the fix (kernels.hpp RING_AHEAD) its
    4th ring slot was not cleared by the 3-sweep launch before it and kept an
    old exact residual, which read as "proven to go on" when above 1. The first
    timestep's source (lid corners only) makes the first iteration fall back;
    with chunk 5 (6) exact launches cover iterations 1..15 (1..18) and the first
    proof launch 16..19 (19..22), whose 4th slot then held the exact residual
    of iteration 3 (6). The source is scaled so that residuals cross the
    reference's primed value 1.0 (cavity-01.cpp:618) around there, and the
    tolerance is placed at the exact residual of each iteration 12..26: every
    solve must equal exact residuals throughout, bit for bit."""
    base = C.make_params("cavity", nx=256, ny=256)
    g = C.CavitySolver(base, ordering="rb", device=0, small_solve="off", tuning=MARCH)
    g.applyBoundaryConditions()
    g.computeTentativeVelocities()
    g.buildSourceTerm()
    f0 = g.field("src").copy()
    g.close()
    srcmax0 = float(np.abs(f0[1:-1, 1:-1]).max())
    res = {}
    for k in (3, 19):
        (_, res[k]), _ = solve_source(C.make_params("cavity", nx=256, ny=256, max_iters=k), f0, False)
    alpha = 0.5 / res[19]  # residual of iteration 19 ~ 0.5 after scaling (SOR is linear in f)
    f = f0 * alpha
    srcmax = srcmax0 * alpha
    r = {}
    for k in range(1, 27):
        (kk, r[k]), _ = solve_source(C.make_params("cavity", nx=256, ny=256, max_iters=k), f, False)
        assert kk == k
    stops = set()
    for k in range(12, 27):
        if not r[k] < 1.0:
            continue
        cp = C.make_params("cavity", nx=256, ny=256)
        cp.tol_factor = r[k] / srcmax * (1.0 + 1e-9)
        for chunk in (5, 6):
            (ie, re_), pe = solve_source(cp, f, False, chunk)
            (ip, rp), pp = solve_source(cp, f, True, chunk)
            assert (ip, rp) == (ie, re_), (k, chunk)
            assert_bits(pp, pe, f"tolerance at iteration {k}, chunk {chunk}")
            stops.add(ie)
    assert len([q for q in stops if 12 <= q <= 26]) >= 3, (stops, r[3], r[19])
