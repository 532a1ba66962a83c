"""Group-phase cycles of the resident red-black solve (diagnostic build with
CFD_RES_STAMPS=1, libcfd_amd_rstamps.so): one warm-up step, then one capped
step; per wave the cycles of its neighbour waits, halo loads, first exchange,
sweeps and group end, summed over the solve; printed per group (mean over the
tiles' waves, and the slowest wave).

usage: CFD_AMD_LIB=libcfd_amd_rstamps.so python3 scripts/dbg/res_stamps.py nx ny [max_iters] [case] [order]
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "computational-fluid-dynamics_amd"))
import numpy as np  # noqa: E402
import cfd_amd as C  # noqa: E402
from cfd_amd import _lib  # noqa: E402

nx, ny = int(sys.argv[1]), int(sys.argv[2])
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 10000
case = sys.argv[4] if len(sys.argv) > 4 else "cavity"
order = sys.argv[5] if len(sys.argv) > 5 else "rb"
cp = C.make_params(case, nx=nx, ny=ny, max_iters=iters)
s = C.solver_for(cp, device=0, ordering=order, small_solve="off", tuning={"resident": 1})
if case == "cavity":
    s.applyBoundaryConditions()
s.step()
s.reset_timing()
s.step()
s.synchronize()
tm = s.timing()
L = _lib.lib()
SEG = 7
n = 256 * 8 * SEG
buf = (ctypes.c_ulonglong * n)()
L.cfd_res_stamps(buf, n)
a = np.frombuffer(buf, dtype=np.uint64).reshape(256, 8, SEG).astype(np.float64)
groups = a[:, :, SEG - 1]
used = groups > 0
names = ["wait", "halo", "first_exchange", "sweeps", "drain", "barrier_flag"]
out = {"case": case, "order": order, "nx": nx, "ny": ny, "iters": iters, "solve_ms": tm.poisson_ms, "launches": tm.poisson_launches,
       "fallbacks": tm.proof_fallbacks, "waves": int(used.sum()),
       "us_per_sweep": 1000 * tm.poisson_ms / iters}
for k, nm in enumerate(names):
    per_group = a[:, :, k][used] / groups[used]
    out[nm + "_cyc_per_group_mean"] = round(float(per_group.mean()), 1)
    out[nm + "_cyc_per_group_max"] = round(float(per_group.max()), 1)
    # per wave index (wave 0 polls; the first / last waves hold the top / bottom halo rows)
    out[nm + "_by_wave"] = [round(float((a[:, w, k][used[:, w]] / groups[:, w][used[:, w]]).mean()), 1)
                            if used[:, w].any() else None for w in range(8)]
# per tile class: the first / last column tiles (ghost columns) vs the others
ctiles = (nx + 2 + 111) // 112
tiles = np.arange(256)
edge = ((tiles % ctiles) == 0) | ((tiles % ctiles) == ctiles - 1)
for nm, k in (("sweeps", 3), ("wait", 0), ("drain", 4), ("barrier_flag", 5)):
    for cls, sel in (("edge_tiles", edge), ("inner_tiles", ~edge)):
        u = used & sel[:, None]
        if u.any():
            out[f"{nm}_{cls}_mean"] = round(float((a[:, :, k][u] / groups[u]).mean()), 1)
tot = sum(a[:, :, k] for k in range(SEG - 1))[used] / groups[used]
out["total_cyc_per_group_mean"] = round(float(tot.mean()), 1)
print(json.dumps(out, indent=1))
