"""BASELINE.json configurations beyond the bench case.

* configs[2] channel flow: the developed profile is Poiseuille (README
  "Validation: parabolic profile"). At Re=1000 on L=3 the flow does not reach
  the developed state (entrance length ~0.05 Re H = 50 H), so the analytic
  check runs at Re=10 (entrance length 0.5 H) to steady state; the Re=1000
  4096x512 grid itself is run for a few steps for shape/health. The
  reference's scheme drains flux along the channel; the CPU
  oracle run of this same case gives flux 0.95287 at x=0.8L, as the GPU does.
* configs[3] backwards step 8192x512 over 4 ranks: 4 rank solvers (loopback
  transport, host threads) against one domain.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import cfd_amd as C  # noqa: E402
from test_gpu_ranks import run_ranks, single  # noqa: E402


def test_channel_poiseuille_profile():
    # viscous development time H^2 / nu = 10: run to t = 25
    cp = C.make_params("channel", re=10.0, nx=96, ny=32, final_time=25.0)
    s = C.ChannelSolver(cp, ordering="rb")
    s.run_steps(cp.total_steps)
    s.statistics()
    uc = s.field("uc")
    y = (np.arange(1, cp.ny + 1) - 0.5) * cp.dy
    exact = 6.0 * y * (1.0 - y)  # mean 1 (inlet velocity), height 1
    i_out = int(0.8 * cp.nx)
    prof = uc[1:cp.ny + 1, i_out]
    # The reference removes the mean of the Poisson source (channel-01.cpp:620-628)
    # even though its outlet is Dirichlet p=0 (line 535), which drains ~5% of
    # the inlet flux at this resolution; the GPU path reproduces that (parity),
    # so the developed profile is checked in shape: u / mean(u) vs 6y(1-y).
    shape = prof / prof.mean()
    dev = np.abs(shape - exact / exact.mean()).max()
    print("flux", prof.mean(), "max |shape - poiseuille| =", dev)
    assert dev <= 0.01 * exact.max(), dev
    assert 0.9 <= prof.mean() <= 1.0 + 1e-9
    # fully developed: the profile shape no longer changes along x downstream
    # (the flux keeps draining linearly, 0.9647 at x=0.6L vs 0.9529 at 0.8L in
    # the CPU oracle too)
    prof2 = uc[1:cp.ny + 1, int(0.6 * cp.nx)]
    assert np.abs(prof2 / prof2.mean() - shape).max() <= 0.01 * exact.max()
    assert prof2.mean() > prof.mean()


def test_channel_re1000_4096x512_runs():
    cp = C.make_params("channel", re=1000.0, nx=4096, ny=512, max_iters=2000)
    s = C.ChannelSolver(cp, ordering="rb")
    for _ in range(3):
        it, res = s.step()
        assert 1 <= it <= cp.max_iters and np.isfinite(res)
    md, ke = s.statistics()
    assert np.isfinite(md) and np.isfinite(ke) and ke > 0


def test_backstep_8192x512_four_ranks():
    cp = C.make_params("backwards_step", re=400.0, nx=8192, ny=512, max_iters=300)
    res = run_ranks(cp, 4, 2)
    s, its = single(cp, 2)
    ref = s.field("u")
    for r in res:
        assert [i for i, _ in r["its"]] == [i for i, _ in its]
        j0, j1 = r["rows"]
        first = 0 if j0 == 1 else j0
        last = j1 + 1 if j1 == cp.ny else j1
        np.testing.assert_allclose(r["u"], ref[first:last + 1], rtol=0, atol=1e-9 * np.abs(ref).max())
