"""The RCCL transport on hardware.

One rank (runs on the 1-GPU box): a torch process set up as bench.py at N>1
builds the communicator via cfd_comm_unique_id / cfd_comm_init (the dlopen'ed
ncclGetUniqueId / ncclCommInitRank), asks RCCL for its size
(cfd_comm_info -> ncclCommCount == 1) and runs the rank-path solver, which
must equal the single-domain solver bit for bit. With one rank the solver
issues NO RCCL collective or send/recv: every halo exchange and all-reduce is
guarded by nranks > 1 (solver.hip). So this checks the bootstrap and the rank
solver's set-up only.

Two ranks on two GPUs (skipped unless two devices are visible): the real data
path — grouped ncclSend/ncclRecv halo exchange, the lagged residual
all-reduce on the second stream, the source-sum / stats all-reduces — each
rank's rows against one domain. The loopback transport
(tests/test_gpu_ranks.py) runs the same rank code on one device."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("case,steps", [("cavity", 5), ("channel", 3)])
def test_one_rank_rccl_equals_single_domain(case, steps):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29611 + (case == "channel")))
    out = subprocess.run([sys.executable, "-u", os.path.join(HERE, "rccl_one_rank.py"), case, str(steps)],
                         env=env, capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["comm"] == {"nranks": 1, "rank": 0, "transport": "rccl"}
    assert d["its"] == d["its_ref"]
    if case == "cavity":
        assert all(d["same"].values()), d


def test_one_rank_rccl_send_recv_to_self():
    """ncclSend / ncclRecv on hardware: the halo exchange's own group
    (comm_halo_exchange) with the one rank as both of its neighbours, on
    halo-sized device buffers (8 rows of a 4096-column strip), one row and one
    double; every received double must equal the sent one bit for bit."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29615")
    out = subprocess.run([sys.executable, "-u", os.path.join(HERE, "rccl_self_exchange.py")],
                         env=env, capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["comm"] == {"nranks": 1, "rank": 0, "transport": "rccl"}
    assert "error" not in d, d
    assert d["mismatches"] == {"32896": 0, "4112": 0, "1": 0}, d


def test_loopback_exchange_check():
    """The same check through the loopback transport (one rank, peer = itself)."""
    import ctypes

    from cfd_amd import _lib
    L = _lib.lib()
    hub = L.cfd_comm_loopback_hub(1)
    comm = L.cfd_comm_init_loopback(hub, 0, 0)
    assert comm, L.cfd_last_error()
    bad = ctypes.c_longlong(-1)
    assert L.cfd_comm_exchange_check(comm, 0, 4112, ctypes.byref(bad)) == 0, L.cfd_last_error()
    assert bad.value == 0
    assert L.cfd_comm_exchange_check(comm, 1, 16, ctypes.byref(bad)) != 0  # (peer outside the communicator)
    L.cfd_comm_destroy(comm)
    L.cfd_comm_loopback_hub_destroy(hub)


def _gpu_count() -> int:
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        return 0


@pytest.mark.skipif(_gpu_count() < 2, reason="needs two GPUs (RCCL refuses two ranks on one device)")
@pytest.mark.parametrize("case,ny,steps", [("cavity", 256, 4), ("channel", 128, 3)])
def test_two_rank_rccl_equals_single_domain(case, ny, steps):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29631 + (case == "channel")))
    out = subprocess.run([sys.executable, "-u", os.path.join(HERE, "rccl_two_ranks.py"), case, str(ny), str(steps)],
                         env=env, capture_output=True, text=True, timeout=200)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["comm"] == [{"nranks": 2, "rank": 0, "transport": "rccl"}, {"nranks": 2, "rank": 1, "transport": "rccl"}]
    assert d["overlapped"] == [True, True]
    assert d["its_equal"], d
    assert d["fields_ok"], d
