"""The RCCL transport on hardware with one rank: a torch process (as bench.py at
N>1) builds the communicator via cfd_comm_unique_id / cfd_comm_init (the
dlopen'ed ncclGetUniqueId / ncclCommInitRank) and runs the rank-path solver,
whose reductions then go through ncclAllReduce. Must equal the single-domain
solver bit for bit. (Halo send/recv needs two devices: left to the driver's
multi-GPU run; its code path is covered by tests/test_gpu_ranks.py.)"""
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
    assert d["its"] == d["its_ref"]
    if case == "cavity":
        assert all(d["same"].values()), d
