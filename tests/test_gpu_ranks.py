"""The multi-process (rank) code path on one GPU: ranks run in host threads of
one process and exchange halos / all-reduce through the library's in-process
loopback transport (RCCL refuses two ranks on one device). Everything but the
RCCL calls themselves is the code the 8-GPU run executes: rank strips, halo
row indices, the residual all-reduce feeding each rank's convergence test,
the source-sum and stats reductions, rank-local field transfer."""
from __future__ import annotations

import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import cfd_amd as C  # noqa: E402
from cfd_amd import _lib  # noqa: E402
from cfd_amd.dist import strip_rows  # noqa: E402


def run_ranks(cp, world, steps, check_every=1, timing=False, **kw):
    L = _lib.lib()
    hub = L.cfd_comm_loopback_hub(world)
    assert hub
    results = [None] * world
    errors = []

    def body(r):
        try:
            comm = L.cfd_comm_init_loopback(hub, r, 0)
            assert comm, L.cfd_last_error()
            s = C.solver_for(cp, ordering="rb", rank_rows=strip_rows(r, world, cp.ny), comm=comm, check_every=check_every, **kw)
            if cp.case_id == C.CAVITY:
                s.applyBoundaryConditions()
            its = [s.step() for _ in range(steps)]
            md, ke = s.statistics()
            results[r] = dict(rows=s.owned_rows(), u=s.field("u"), v=s.field("v"), p=s.field("p"), its=its,
                              stats=(md, ke), overlapped=s.timing().poisson_overlapped,
                              fallbacks=s.timing().proof_fallbacks)
            s.close()
            L.cfd_comm_destroy(comm)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    L.cfd_comm_loopback_hub_destroy(hub)
    assert not errors, errors
    return results


def single(cp, steps, **kw):
    s = C.solver_for(cp, ordering="rb", **kw)
    if cp.case_id == C.CAVITY:
        s.applyBoundaryConditions()
    its = [s.step() for _ in range(steps)]
    return s, its


@pytest.mark.parametrize("case,world,steps", [("cavity", 2, 15), ("cavity", 3, 10), ("channel", 2, 10),
                                               ("backwards_step", 2, 2)])
def test_rank_path_equals_single_domain(case, world, steps):
    cp = C.reference_defaults(case)
    res = run_ranks(cp, world, steps)
    s, its = single(cp, steps)
    ref = {n: s.field(n) for n in ("u", "v", "p")}
    for r in res:
        if case == "cavity":
            assert r["its"] == its
        else:
            assert [i for i, _ in r["its"]] == [i for i, _ in its]
        j0, j1 = r["rows"]
        first = 0 if j0 == 1 else j0
        for n in ("u", "v", "p"):
            rows_total = ref[n].shape[0]
            last = min(j1 + 1 if j1 == cp.ny else j1, rows_total - 1)
            a, b = r[n], ref[n][first:last + 1]
            if case == "cavity":
                assert np.array_equal(a.view(np.int64), b.view(np.int64)), (n, r["rows"])
            else:
                np.testing.assert_allclose(a, b, rtol=0, atol=1e-9 * max(np.abs(b).max(), 1.0))
    md, ke = s.statistics()
    for r in res:
        if case == "cavity":
            assert r["stats"][0] == md
        else:  # source mean summed per rank then all-reduced: re-associated
            assert r["stats"][0] == pytest.approx(md, rel=1e-9)
        assert r["stats"][1] == pytest.approx(ke, rel=1e-12)


def test_rank_path_check_every_8():
    """check_every=8 (an option; every GPU count defaults to 1, the reference's
    rule): the solve may run up to 7 sweeps past the reference's stopping
    point, never fewer, and still converges."""
    cp = C.reference_defaults("cavity")
    res = run_ranks(cp, 2, 5, check_every=8)
    _, its = single(cp, 5)
    for r in res:
        for (ig, rg), (i1, _r1) in zip(r["its"], its):
            assert i1 <= ig <= i1 + 7
            assert ig % 8 == 0 or ig == cp.max_iters


@pytest.mark.parametrize("case,world,ny,steps", [("cavity", 2, 128, 6), ("cavity", 3, 160, 4), ("channel", 2, 128, 4)])
def test_overlapped_halo_exchange_equals_single_domain(case, world, ny, steps):
    """Strips of >= 48 rows split each pair launch: the rows within 16 of a
    neighbour (after the halo exchange) on a second stream, the interior rows
    concurrently on the first. Must equal one domain (cavity bit for bit)."""
    cp = C.make_params(case, ny=ny, nx=96)
    res = run_ranks(cp, world, steps)
    s, its = single(cp, steps)
    ref = {n: s.field(n) for n in ("u", "v", "p")}
    for r in res:
        assert r["overlapped"] > 0, "overlap path not taken"
        if case == "cavity":
            assert r["its"] == its
        else:
            assert [i for i, _ in r["its"]] == [i for i, _ in its]
        j0, j1 = r["rows"]
        first = 0 if j0 == 1 else j0
        for n in ("u", "v", "p"):
            last = min(j1 + 1 if j1 == cp.ny else j1, ref[n].shape[0] - 1)
            a, b = r[n], ref[n][first:last + 1]
            if case == "cavity":
                assert np.array_equal(a.view(np.int64), b.view(np.int64)), (n, r["rows"])
            else:
                np.testing.assert_allclose(a, b, rtol=0, atol=1e-9 * max(np.abs(b).max(), 1.0))


@pytest.mark.parametrize("delta", [-2, -1, 0, 1, 2, 3])
def test_overlapped_lagged_stop_and_caps(delta):
    """Overlapped ranks test the residuals one pair late (their all-reduce runs
    beside the next launch) and keep three pressure buffers: a stop at an odd
    or even count, a cap just below / at / above the natural stop K, and the
    host's test of the last untested iterations must all give the
    single-domain iteration count and field."""
    base = C.make_params("cavity", ny=128, nx=96)
    s0, its0 = single(base, 1)
    K = its0[0][0]
    cp = C.make_params("cavity", ny=128, nx=96, max_iters=max(1, K + delta))
    res = run_ranks(cp, 2, 2)
    s, its = single(cp, 2)
    ref = s.field("p")
    for r in res:
        assert r["overlapped"] > 0
        assert r["its"] == its, (K, delta)
        j0, j1 = r["rows"]
        first = 0 if j0 == 1 else j0
        last = min(j1 + 1 if j1 == cp.ny else j1, ref.shape[0] - 1)
        assert np.array_equal(r["p"].view(np.int64), ref[first:last + 1].view(np.int64))


@pytest.mark.parametrize("world,nx,ny,steps,cap", [(2, 256, 256, 3, 0), (3, 300, 240, 2, 0), (2, 512, 512, 2, 61)])
def test_proof_mode_on_ranks(world, nx, ny, steps, cap):
    """The proof-mode convergence test on ranks: interior column
    tiles (nx >= 240), overlapped strips with the lagged test, ratios
    all-reduced (max) like residuals. Iteration counts and fields must equal
    one domain with exact residuals, bit for bit."""
    kw = {"max_iters": cap} if cap else {}
    cp = C.make_params("cavity", nx=nx, ny=ny, **kw)
    s, its = single(cp, steps, small_solve="off", proof_test="off")
    ref = s.field("p")
    res = run_ranks(cp, world, steps, proof_test="on")
    for r in res:
        assert r["overlapped"] > 0
        assert r["its"] == its
        if cap:
            assert r["fallbacks"] == 1  # the first step's corner-only source (tests/test_gpu_proof.py)
        else:
            assert r["fallbacks"] >= sum(1 for k, _ in its if k < cp.max_iters)
        j0, j1 = r["rows"]
        first = 0 if j0 == 1 else j0
        last = min(j1 + 1 if j1 == cp.ny else j1, ref.shape[0] - 1)
        assert np.array_equal(r["p"].view(np.int64), ref[first:last + 1].view(np.int64))


@pytest.mark.parametrize("case,world,nx,ny,steps,cap", [("channel", 2, 300, 160, 3, 0), ("channel", 3, 256, 200, 2, 900),
                                                        ("backwards_step", 2, 400, 160, 2, 0),
                                                        ("backwards_step", 4, 512, 256, 2, 700)])
def test_open_proof_mode_on_ranks(case, world, nx, ny, steps, cap):
    """The open cases' proof-mode launches (open.hip: 4 sweeps for the
    channel, 3 for the step on ranks) on overlapped ranks with the lagged,
    all-reduced test, against one domain with exact residuals: iteration
    counts equal; fields to 1e-9 (the source's mean removal is summed per rank
    and all-reduced, a re-association)."""
    kw = {"max_iters": cap} if cap else {}
    cp = C.make_params(case, nx=nx, ny=ny, **kw)
    s, its = single(cp, steps, small_solve="off", proof_test="off", tuning={"tile_rounds": 0, "resident": 0})
    ref = {n: s.field(n) for n in ("u", "v", "p")}
    res = run_ranks(cp, world, steps, proof_test="on")
    for r in res:
        assert r["overlapped"] > 0
        assert [i for i, _ in r["its"]] == [i for i, _ in its]
        j0, j1 = r["rows"]
        first = 0 if j0 == 1 else j0
        for n in ("u", "v", "p"):
            last = min(j1 + 1 if j1 == cp.ny else j1, ref[n].shape[0] - 1)
            a, b = r[n], ref[n][first:last + 1]
            np.testing.assert_allclose(a, b, rtol=0, atol=1e-9 * max(np.abs(b).max(), 1.0))
