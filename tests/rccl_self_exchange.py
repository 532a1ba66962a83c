"""Child process of tests/test_gpu_rccl.py: the halo exchange's send / recv
group (comm.hip comm_halo_exchange, the call sites Solver::exchange uses) on a
one-rank RCCL communicator whose rank is its own neighbour below and above
(ncclSend / ncclRecv to self, inside ncclGroupStart / ncclGroupEnd), on
device buffers the size of a 4096-column strip's 8-row halo and of one row.
Prints one JSON line: the communicator info and the mismatch count per size."""
import ctypes
import json
import os
import sys

import torch  # noqa: F401  (first: the library binds to PyTorch's HIP runtime, as in bench.py)
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "computational-fluid-dynamics_amd"))
from cfd_amd import _lib  # noqa: E402
from cfd_amd.dist import comm_info, init_comm  # noqa: E402


def main() -> int:
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=0, world_size=1)
    comm = init_comm(dist, 0, 1, 0)
    out = {"comm": comm_info(comm), "mismatches": {}}
    pitch = (4096 + 3 + 15) // 16 * 16  # (the 4096-column slab's row pitch)
    for count in (8 * pitch, pitch, 1):
        bad = ctypes.c_longlong(-1)
        rc = _lib.lib().cfd_comm_exchange_check(comm, 0, count, ctypes.byref(bad))
        if rc != 0:
            out["error"] = _lib.lib().cfd_last_error().decode(errors="replace")
            break
        out["mismatches"][str(count)] = bad.value
    _lib.lib().cfd_comm_destroy(comm)
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
