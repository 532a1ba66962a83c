"""Child process of tests/test_gpu_rccl.py: the bench's multi-GPU set-up
(torch first, gloo process group, RCCL communicator through the library's
dlopen table) with one rank. With one rank the solver issues no RCCL
collective (all are guarded by nranks > 1); this checks the bootstrap, RCCL's
own view of the communicator (ncclCommCount / ncclCommUserRank) and the rank
solver. Prints one JSON line: the communicator info, the rank solver's SOR
counts and whether its fields equal the single-domain solver's bit for bit."""
import json
import os
import sys

import torch  # noqa: F401  (first: the library binds to PyTorch's HIP runtime, as in bench.py)
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "computational-fluid-dynamics_amd"))
import numpy as np  # noqa: E402

import cfd_amd as C  # noqa: E402
from cfd_amd import _lib  # noqa: E402
from cfd_amd.dist import comm_info, init_comm, strip_rows  # noqa: E402


def main() -> int:
    case, steps = sys.argv[1], int(sys.argv[2])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=0, world_size=1)
    comm = init_comm(dist, 0, 1, 0)
    info = comm_info(comm)
    cp = C.reference_defaults(case)
    s = C.solver_for(cp, ordering="rb", rank_rows=strip_rows(0, 1, cp.ny), comm=comm, check_every=1)
    if case == "cavity":
        s.applyBoundaryConditions()
    its = [s.step() for _ in range(steps)]
    fields = {n: s.field(n) for n in ("u", "v", "p")}
    s.close()
    _lib.lib().cfd_comm_destroy(comm)

    r = C.solver_for(cp, ordering="rb")
    if case == "cavity":
        r.applyBoundaryConditions()
    its_ref = [r.step() for _ in range(steps)]
    same = {n: bool(np.array_equal(fields[n].view(np.int64), r.field(n).view(np.int64))) for n in fields}
    r.close()
    dist.destroy_process_group()
    print(json.dumps({"comm": info, "its": [int(i) for i, _ in its], "its_ref": [int(i) for i, _ in its_ref], "same": same}),
          flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
