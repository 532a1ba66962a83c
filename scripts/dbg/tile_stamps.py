"""Phase shares of the LDS-tile SOR launch (diagnostic build with
CFD_TILE_STAMPS=1, libcfd_amd_stamps.so): one capped step of a workload,
then the last tile launch's per-wave shader-clock sums per phase, averaged
over the waves / blocks that ran. Shares only: the stamps' waits forbid
overlaps the product kernel has.

usage: CFD_AMD_LIB=libcfd_amd_stamps.so python3 scripts/dbg/tile_stamps.py case nx ny [max_iters]
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "computational-fluid-dynamics_amd"))
import numpy as np  # noqa: E402
import cfd_amd as C  # noqa: E402
from cfd_amd import _lib  # noqa: E402

SEGS = ["load", "red", "red_barrier", "black", "black_barrier", "refresh", "residual", "store"]
case, nx, ny = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 400
cp = C.make_params(case, nx=nx, ny=ny, max_iters=iters)
s = C.solver_for(cp, device=0, ordering="rb")  # (the tile launches: red-black order)
s.step()
s.synchronize()
t = s.timing()
L = _lib.lib()
n = 1024 * 16 * 8
buf = (ctypes.c_ulonglong * n)()
got = L.cfd_tile_stamps(buf, n)
a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 16, 8).astype(np.float64)
ran = a.sum(axis=2) > 0
blocks = int(ran.any(axis=1).sum())
mean = a[ran].mean(axis=0)
tot = mean.sum()
out = {"case": case, "nx": nx, "ny": ny, "sor_kernel": int(t.sor_kernel), "blocks": blocks,
       "cycles_per_wave": round(float(tot)),
       "share": {k: round(float(v / tot), 4) for k, v in zip(SEGS, mean)},
       "cycles": {k: round(float(v)) for k, v in zip(SEGS, mean)},
       "max_over_waves_cycles": {k: round(float(v)) for k, v in zip(SEGS, a[ran].max(axis=0))}}
print(json.dumps(out))
s.close()
