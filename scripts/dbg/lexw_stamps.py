"""Per-launch march durations of the reference-order solve (diagnostic build
with CFD_LEXW_STAMPS=1, libcfd_amd_lstamps.so): one capped timestep, then for
every launch (H0 / 2NS) and march path the slowest wave's cycles, the mean and
the wave count; printed as a summary over the ramp-up, steady and ramp-down
launches.

usage: CFD_AMD_LIB=libcfd_amd_lstamps.so python3 scripts/dbg/lexw_stamps.py case nx ny [max_iters] [knob=value ...]
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "computational-fluid-dynamics_amd"))
import numpy as np  # noqa: E402
import cfd_amd as C  # noqa: E402
from cfd_amd import _lib  # noqa: E402

PATHS = ["wall", "ramp_full", "ramp_masked", "steady", "step_block", "step_left", "ramp_masked_rc", "steady_rc"]
case, nx, ny = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 10000
tuning = {k: int(v) for k, v in (a.split("=") for a in sys.argv[5:])}
cp = C.make_params(case, nx=nx, ny=ny, max_iters=iters, **({"re": 400.0} if case == "backwards_step" else {}))
s = C.solver_for(cp, device=0, ordering="lex", tuning=tuning)
s.step()
s.synchronize()
L = _lib.lib()
n = 8192 * 8 * 3
buf = (ctypes.c_ulonglong * n)()
L.cfd_lexw_stamps(buf, n)
a = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 8, 3).astype(np.float64)
used = a[:, :, 2].sum(axis=1) > 0
idx = np.nonzero(used)[0]
launch_max = a[:, :, 0].max(axis=1)
out = {"case": case, "nx": nx, "ny": ny, "launches": int(len(idx))}
# the slowest path per launch, and the launch-max distribution in launch-index tenths
tenths = np.array_split(idx, 10)
rows = []
for part in tenths:
    if len(part) == 0:
        continue
    lm = launch_max[part]
    slow = a[part, :, 0].argmax(axis=1)
    kinds = {PATHS[k]: int((slow == k).sum()) for k in set(slow.tolist())}
    per_path = {}
    for k in range(8):
        w = a[part, k, 2].sum()
        if w > 0:
            per_path[PATHS[k]] = {"waves_per_launch": round(float(w / len(part)), 1),
                                  "mean_cycles": round(float(a[part, k, 1].sum() / w)),
                                  "max_cycles_mean": round(float(a[part, k, 0][a[part, k, 2] > 0].mean()))}
    rows.append({"launches": [int(part[0]), int(part[-1])], "launch_max_cycles_mean": round(float(lm.mean())),
                 "slowest_path": kinds, "paths": per_path})
out["by_tenth"] = rows
print(json.dumps(out, indent=1))
s.close()
