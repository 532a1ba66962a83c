"""Per-wave march durations of the open cases' proof launch (diagnostic build
with CFD_OPEN_STAMPS=1, libcfd_amd_ostamps.so): one capped step, then the
last launch's waves grouped by path (interior columns / safe band / edge
masks) and column class (left of the step's column, across it, right).

usage: CFD_AMD_LIB=libcfd_amd_ostamps.so python3 scripts/dbg/open_stamps.py case nx ny [max_iters]
(CFD_STAMPS_FN=cfd_march_stamps with a CFD_MARCH_STAMPS=1 build: the cavity /
pair march, poisson_multi_kernel)
"""
import collections
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "computational-fluid-dynamics_amd"))
import numpy as np  # noqa: E402
import cfd_amd as C  # noqa: E402
from cfd_amd import _lib  # noqa: E402

case, nx, ny = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 400
cp = C.make_params(case, nx=nx, ny=ny, max_iters=iters)
s = C.solver_for(cp, device=0, ordering="rb")  # (the proof launches: red-black order)
s.step()
s.synchronize()
L = _lib.lib()
n = 8192 * 8
buf = (ctypes.c_longlong * n)()
getattr(L, os.environ.get("CFD_STAMPS_FN", "cfd_open_stamps"))(buf, n)
a = np.frombuffer(buf, dtype=np.int64).reshape(8192, 8)
a = a[a[:, 7] > 0]
step_i = getattr(cp, "step_i", 0) if case == "backwards_step" else -1
groups = collections.defaultdict(list)
for tile, ct, band, y0, y1, cin, safe, cyc in a.tolist():
    c0 = ct * 112 - 8
    col = "left" if (step_i > 0 and c0 + 127 <= step_i - 1) else \
          "across" if (step_i > 0 and not c0 > step_i + 1) else "right"
    path = "safe" if safe else ("interior_cols" if cin else "edge")
    groups[(col, path, y1 - y0)].append(cyc)
rows = []
for k, v in sorted(groups.items()):
    rows.append({"cols": k[0], "path": k[1], "band_rows": k[2], "waves": len(v),
                 "mean_cycles": int(np.mean(v)), "max_cycles": int(np.max(v))})
top = a[np.argsort(-a[:, 7])[:12]].tolist()
print(json.dumps({"case": case, "nx": nx, "ny": ny, "waves": int(len(a)), "groups": rows,
                  "slowest": [dict(zip(["tile", "ctile", "band", "y0", "y1", "cols_in", "safe", "cycles"], t))
                              for t in top]}, indent=1))
s.close()
