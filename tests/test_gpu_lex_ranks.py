"""The reference's own sweep order on ranks (ABI 12), bit for bit.

Ranks are host threads of one process sharing the GPU over the library's
loopback transport (the same group send / recv / all-reduce call sites as
RCCL; RCCL refuses two ranks on one device). Each rank runs the multi-block
reference-order march (csrc/lexw.hpp) on its strip with the 8-row halos
exchanged before every launch; the stop rule's per-iteration exceedance bits
are OR-ed over the ranks (a max all-reduce) before the launches that test
them; the open cases' source sum and the kinetic energy are one sequential
chain rank to rank (Solver::seq_sum_ranks). So every iteration count,
residual and field must equal the oracle's restatement of the reference
loop (ORC_LEX, pinned to the reference binaries by test_oracle_golden.py)
and one device, bit for bit, at every rank count.

Reference loops: cavity-01.cpp:635-678, channel-01.cpp:620-628 (mean) and
:652-668, backwards_step-01.cpp:843-862 (mean) and :893-939 (SOR).
"""
from __future__ import annotations

import hashlib
import json
import os
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import cfd_amd as C  # noqa: E402
import oracle as O  # noqa: E402
from cfd_amd import _lib  # noqa: E402
from cfd_amd.dist import strip_rows  # noqa: E402
from test_gpu_parity import assert_bits, ofield  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lex_digests.json")
FIELDS = ("u", "v", "p")


def run_lex_ranks(cp, world, steps, stats=True, **kw):
    """`steps` whole timesteps on `world` loopback ranks in the reference's
    order; per rank: its rows, fields, (iterations, residual) per step, stats,
    timing."""
    L = _lib.lib()
    hub = L.cfd_comm_loopback_hub(world)
    assert hub
    results = [None] * world
    errors = []

    def body(r):
        try:
            comm = L.cfd_comm_init_loopback(hub, r, 0)
            assert comm, L.cfd_last_error()
            s = C.solver_for(cp, ordering="lex", rank_rows=strip_rows(r, world, cp.ny), comm=comm, **kw)
            if cp.case_id == C.CAVITY:
                s.applyBoundaryConditions()
            its = [s.step() for _ in range(steps)]
            st = s.statistics() if stats else None
            tm = s.timing()
            results[r] = dict(rows=s.owned_rows(), its=its, stats=st, **{n: s.field(n) for n in FIELDS},
                              kernel=_lib.SOR_KERNEL.get(tm.sor_kernel), steady=tm.poisson_steady_launches,
                              fallbacks=tm.proof_fallbacks)
            s.close()
            L.cfd_comm_destroy(comm)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=900)
    L.cfd_comm_loopback_hub_destroy(hub)
    assert not errors, errors
    return results


def assemble(res, name, cp):
    """The global field from the ranks' owned rows (rank 0 holds ghost row 0,
    the last rank the top ghost row)."""
    return np.concatenate([r[name] for r in res], axis=0)


def oracle_run(cp, steps):
    o = O.Oracle(cp, ordering=O.LEX)
    o.velocity_bc(False)  # cavity: the step's first BC is idempotent; open cases: the constructor's BC
    its = [o.step() for _ in range(steps)]
    return o, its


@pytest.mark.parametrize("case,world,steps", [("cavity", 2, 6), ("cavity", 4, 4), ("channel", 3, 4),
                                               ("backwards_step", 2, 2), ("backwards_step", 4, 2)])
def test_reference_defaults_on_ranks_equal_oracle(case, world, steps):
    """The reference's own runs (63^2 cavity, 93x31 channel, 256x32 step): the
    cavity and channel solves converge (stop found on the all-reduced bits,
    replayed to the reference's count), the step's hit the cap."""
    cp = C.reference_defaults(case)
    res = run_lex_ranks(cp, world, steps)
    o, its = oracle_run(cp, steps)
    for r in res:
        assert r["kernel"] == "lexw"
        assert r["its"] == its, r["rows"]
    for name in FIELDS:
        assert_bits(assemble(res, name, cp), ofield(o, name, cp), f"{case} {world} ranks {name}")
    o.centers()
    md, ke = o.stats()
    for r in res:
        assert r["stats"] == (md, ke)


@pytest.mark.parametrize("world", [2, 3, 4])
def test_capped_cavity_on_ranks_equal_oracle(world):
    """Capped solves past (nx+ny)/2: every rank runs steady launches between
    its ramps."""
    cp = C.make_params("cavity", nx=200, ny=160, max_iters=260)
    res = run_lex_ranks(cp, world, 2)
    o, its = oracle_run(cp, 2)
    for r in res:
        assert r["its"] == its
        assert r["steady"] > 0
    for name in FIELDS:
        assert_bits(assemble(res, name, cp), ofield(o, name, cp), f"cavity capped {world} ranks {name}")


def test_tall_grid_per_strip_steady_windows():
    """nx + ny > 2K: the whole grid never has a launch with every cell active,
    but each 128-row strip does (Solver::run_lexw's per-strip window)."""
    cp = C.make_params("cavity", nx=64, ny=512, max_iters=220)
    res = run_lex_ranks(cp, 4, 1)
    o, its = oracle_run(cp, 1)
    assert all(r["steady"] > 0 for r in res)
    for r in res:
        assert r["its"] == its
    for name in FIELDS:
        assert_bits(assemble(res, name, cp), ofield(o, name, cp), f"tall {name}")


@pytest.mark.parametrize("case,world,nx,ny,K", [("channel", 2, 300, 96, 160), ("channel", 4, 256, 128, 200),
                                                ("backwards_step", 3, 320, 96, 120),
                                                ("backwards_step", 4, 400, 128, 230)])
def test_open_cases_on_ranks_equal_oracle(case, world, nx, ny, K):
    """Channel and step: the source mean is one sequential sum chained rank
    to rank, the ghost / solid refresh in the skew crosses the rank edges
    (the step's block edge lies inside a rank or on a rank edge)."""
    cp = C.make_params(case, nx=nx, ny=ny, max_iters=K)
    res = run_lex_ranks(cp, world, 2)
    o, its = oracle_run(cp, 2)
    for r in res:
        assert r["its"] == its
    for name in FIELDS:
        assert_bits(assemble(res, name, cp), ofield(o, name, cp), f"{case} {world} ranks {name}")
    o.centers()
    assert res[0]["stats"] == o.stats()


def test_ranks_equal_one_device_and_strips():
    """The same grid on one device, on 3 strips of one device and on 3 ranks:
    identical bits (the decomposition never changes the result)."""
    cp = C.make_params("channel", nx=240, ny=120, max_iters=300)
    res = run_lex_ranks(cp, 3, 2)
    for strips in (1, 3):
        g = C.ChannelSolver(cp, ordering="lex", small_solve="off", n_strips=strips, tuning={"resident": 0})
        its = [g.step() for _ in range(2)]
        assert res[0]["its"] == its
        for name in FIELDS:
            assert_bits(assemble(res, name, cp), g.field(name), f"strips={strips} {name}")
        assert res[1]["stats"] == g.statistics()
        g.close()


def _digest(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<f8").tobytes()).hexdigest()


def test_config3_backstep_8192x512_four_ranks_digest():
    """BASELINE configs[3] as stated: the backwards step at 8192x512 on four
    ranks (8192x128 each), one capped timestep with K = 4400 in the
    reference's order, against the oracle's digest of the same step
    (tests/golden/make_lex_digests.py): iteration count, residual and the
    sha256 of u, v, p."""
    d = json.load(open(GOLDEN))["backwards_step_8192x512_K4400"]
    kw = dict(d["params"])
    case = kw.pop("case")
    cp = C.make_params(case, **kw)
    res = run_lex_ranks(cp, 4, 1, stats=False)
    for r in res:
        assert r["its"][0][0] == d["sor_iterations"]
        assert r["its"][0][1].hex() == d["residual"]
        assert r["steady"] > 0
    got = {n: _digest(assemble(res, n, cp)) for n in FIELDS}
    assert got == d["sha256"]
