"""The one-workgroup LDS solve (small.hpp) used for reference-sized grids:
whole timesteps bit-exact against the oracle's red-black restatement and
against the multi-launch kernels (small_solve="off") on the reference's own grids
(cavity 63², channel 93x31, step 256x32) and BASELINE configs[0] (128²) —
the open cases against the oracle to 1e-8 (their source mean is re-associated)
and bit-exact against the multi-launch path — the
stop rule with check_every > 1, and the size limit (a grid just over it takes
the multi-launch path with the same results)."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import cfd_amd as C  # noqa: E402
import oracle as O  # noqa: E402
from test_gpu_parity import assert_bits, ofield  # noqa: E402


def run_gpu(cp, steps, small=True, cavity=True, **kw):
    g = C.solver_for(cp, ordering="rb", small_solve="on" if small else "off", **kw)
    if cavity:  # cavity-01.cpp:380 (the open cases apply their BCs in the constructor)
        g.applyBoundaryConditions()
    its = [g.step() for _ in range(steps)]
    fields = {n: g.field(n).copy() for n in ("u", "v", "p")}
    tm = g.timing()
    g.close()
    return its, fields, tm


@pytest.mark.parametrize("case,kw,steps", [
    ("cavity", {}, 25),
    ("channel", {}, 25),
    ("backwards_step", {}, 25),
    ("cavity", {"re": 100.0, "nx": 128, "ny": 128, "dt": 1e-3}, 10),
])
def test_small_solve_bitexact_vs_oracle_and_multi_launch(case, kw, steps):
    cp = C.reference_defaults(case) if not kw else C.make_params(case, **kw)
    assert (cp.nx + 2) * (cp.ny + 2) <= 20224
    cav = case == "cavity"
    its_s, f_s, tm = run_gpu(cp, steps, small=True, cavity=cav)
    assert tm.poisson_launches == steps  # one launch per solve: the small path ran
    o = O.Oracle(cp, ordering=O.RB)
    if case != "cavity":
        o.velocity_bc(False)
    its_o = [o.step() for _ in range(steps)]
    if cav:  # bit-exact
        assert its_s == its_o
        for n in ("u", "v", "p"):
            assert_bits(f_s[n], ofield(o, n, cp), f"{case} small vs oracle {n}")
    else:  # the source's mean is a tree sum on the GPU, a sequential one in the oracle
        assert [i for i, _ in its_s] == [i for i, _ in its_o]
        for n in ("u", "v", "p"):
            ref = ofield(o, n, cp)
            np.testing.assert_allclose(f_s[n], ref, rtol=0, atol=1e-8 * np.abs(ref).max(), err_msg=n)
    its_m, f_m, tm_m = run_gpu(cp, steps, small=False, cavity=cav)
    assert tm_m.poisson_launches > steps
    assert its_m == its_s
    for n in ("u", "v", "p"):
        assert_bits(f_s[n], f_m[n], f"{case} small vs multi-launch {n}")


def test_small_check_every_and_cap():
    cp = C.make_params("cavity", nx=48, ny=40, max_iters=57)
    its_s, f_s, _ = run_gpu(cp, 6, small=True, check_every=4)
    its_m, f_m, _ = run_gpu(cp, 6, small=False, check_every=4)
    assert its_s == its_m
    assert any(i == 57 for i, _ in its_s) or all(i % 4 == 0 for i, _ in its_s)
    assert_bits(f_s["p"], f_m["p"], "check_every 4")


def test_over_the_limit_takes_multi_launch():
    cp = C.make_params("cavity", nx=150, ny=150, max_iters=200)  # 152² > 20224
    its, _, tm = run_gpu(cp, 2, small=True)
    assert tm.poisson_launches > 2
