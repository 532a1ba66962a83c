"""Several SOR iterations per launch (poisson_multi_kernel: 2, or 3 for the
cavity) against one per launch (poisson_wave_kernel): the fused launch must be
invisible — same iteration counts, same residuals, same fields, bit for bit —
including the edge cases of the launch plan (csrc/solver.hip, Solver::solve):

* a solve that stops inside a launch (the launch already computed further;
  the host replays the first r of its iterations from the launch's input);
* an iteration cap that leaves a shorter last launch, or whose last
  iterations no launch tested (tested on the host after the loop);
* row strips (8-row halos exchanged once per launch) and check_every > 1.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import cfd_amd as C  # noqa: E402
import oracle as O  # noqa: E402
from test_gpu_parity import assert_bits  # noqa: E402



# These are tests of the wave-march launch plan: reference-sized grids would
# otherwise take the one-workgroup solve (small.hpp, tests/test_gpu_small.py)
# or the LDS-tile launches (tile.hpp, tests/test_gpu_tile.py).
MULTI = {"small_solve": "off", "tuning": {"tile_rounds": 0, "resident": 0}}


SOLVERS = {"cavity": C.CavitySolver, "channel": C.ChannelSolver, "backwards_step": C.BackwardsStepSolver}
FIELDS = ("p", "u", "v")


def run(case, cp, steps, **kw):
    g = SOLVERS[case](cp, ordering="rb", device=0, **MULTI, **kw)
    hist = [g.step() for _ in range(steps)]
    out = {n: g.field(n).copy() for n in FIELDS}
    tm = g.timing()
    g.close()
    return hist, out, tm


@pytest.mark.parametrize("case,spl", [("cavity", 2), ("cavity", 3), ("cavity", 0), ("channel", 2), ("channel", 0),
                                      ("backwards_step", 2)])
def test_pairs_equal_single_sweeps(case, spl):
    cp = C.reference_defaults(case)
    steps = 6 if case != "backwards_step" else 2
    h1, f1, t1 = run(case, cp, steps, sweeps_per_launch=1)
    h2, f2, t2 = run(case, cp, steps, sweeps_per_launch=spl)
    assert h1 == h2
    for n in FIELDS:
        assert_bits(f2[n], f1[n], f"{case} {n}")
    assert t2.poisson_launches < t1.poisson_launches  # the fused path really ran
    assert t1.poisson_sweeps == t1.poisson_launches


@pytest.mark.parametrize("spl", [2, 3])
def test_stop_inside_a_launch_is_replayed_and_matches_oracle(spl):
    cp = C.reference_defaults("cavity")
    g = C.CavitySolver(cp, ordering="rb", device=0, sweeps_per_launch=spl, **MULTI)
    o = O.Oracle(cp, ordering=O.RB)
    it_g, res_g = g.step()
    it_o, res_o = o.step()
    assert (it_g, res_g) == (it_o, res_o)
    r = it_g % spl  # iterations of the stopping launch that count
    assert r != 0, "fixture meant to stop inside a launch (replay path)"
    tm = g.timing()
    full = (it_g - r) // spl + 1  # launches up to the stopping one
    assert tm.poisson_launches == full + 1  # ... then one replay launch
    assert tm.poisson_sweeps == full * spl + r
    assert_bits(g.field("p"), o.field("p"), "p after a stop inside a launch")
    g.close()


@pytest.mark.parametrize("spl", [2, 3])
@pytest.mark.parametrize("delta", [-2, -1, 0, 1, 2, 3])
def test_iteration_cap_edges(spl, delta):
    """cap = K + delta around the natural stop K: caps below K (not converged,
    shorter last launches), at K, and above K (the stop found by a launch, or
    by the host's test of the iterations no launch tested)."""
    base = C.reference_defaults("cavity")
    K, _ = C.CavitySolver(base, ordering="rb", device=0, sweeps_per_launch=1, **MULTI).step()
    cp = C.make_params("cavity", max_iters=K + delta)
    h1, f1, _ = run("cavity", cp, 1, sweeps_per_launch=1)
    h2, f2, _ = run("cavity", cp, 1, sweeps_per_launch=spl)
    assert h1 == h2
    assert h1[0][0] == min(K, K + delta)
    assert_bits(f2["p"], f1["p"], f"p cap K{delta:+d}")


@pytest.mark.parametrize("case", ["cavity", "channel"])
@pytest.mark.parametrize("check_every", [1, 8])
def test_pairs_on_strips(case, check_every):
    cp = C.reference_defaults(case)
    h1, f1, _ = run(case, cp, 3, sweeps_per_launch=1, check_every=check_every)
    h2, f2, _ = run(case, cp, 3, sweeps_per_launch=0, check_every=check_every, n_strips=3)
    assert [k for k, _ in h1] == [k for k, _ in h2]
    tol = 0.0 if case == "cavity" else 1e-12
    for n in FIELDS:
        if tol == 0.0:
            assert_bits(f2[n], f1[n], f"{case} {n}")
        else:
            np.testing.assert_allclose(f2[n], f1[n], rtol=0, atol=tol * max(1.0, np.abs(f1[n]).max()))


@pytest.mark.parametrize("spl", [2, 3])
def test_pairs_full_size_bitexact(spl):
    """BASELINE configs[1] size (4096^2): 31 sweeps (15 pairs + 1 single, or 10
    triples + 1 single) == 31 single launches, bit for bit."""
    cp = C.make_params("cavity", nx=4096, ny=4096, max_iters=31)
    h1, f1, _ = run("cavity", cp, 1, sweeps_per_launch=1)
    h2, f2, _ = run("cavity", cp, 1, sweeps_per_launch=spl)
    assert h1 == h2 and h1[0][0] == 31
    assert_bits(f2["p"], f1["p"], "p 4096^2")
