"""Per-wave march cycles of 8 consecutive steady reference-order launches
(diagnostic build CFD_LEXW_STAMPS=1): is the launch set by waves that are
slow in every launch (a persistent imbalance) or by random stragglers?
usage: CFD_AMD_LIB=libcfd_amd_lstamps.so python3 scripts/dbg/lexw_wstamps.py [nx ny]"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "computational-fluid-dynamics_amd"))
import numpy as np  # noqa: E402
import cfd_amd as C  # noqa: E402
from cfd_amd import _lib  # noqa: E402

nx = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
ny = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
cp = C.make_params("cavity", nx=nx, ny=ny, max_iters=10000)
s = C.solver_for(cp, device=0, ordering="lex")
s.applyBoundaryConditions()
s.step()
s.synchronize()
L = _lib.lib()
N, T = 8, 4096
buf = (ctypes.c_ulonglong * (N * T * 4))()
L.cfd_lexw_wstamps.restype = ctypes.c_int
L.cfd_lexw_wstamps(buf, N * T * 4)
a = np.frombuffer(buf, dtype=np.uint64).reshape(N, T, 4)
cyc = a[:, :, 0].astype(np.float64)
used = (cyc > 0).all(axis=0)
cyc = cyc[:, used]
start = a[:, used, 1].astype(np.float64)
ct = (a[0, used, 2] >> 32).astype(int)
y0 = (a[0, used, 2] & 0xffffffff).astype(int)
xcc = a[0, used, 3].astype(int)
out = {"waves": int(used.sum()), "launch_mean": cyc.mean(axis=1).tolist(), "launch_max": cyc.max(axis=1).tolist(),
       "start_spread": (start.max(axis=1) - start.min(axis=1)).tolist()}
# correlation of a wave's cycles between launches (persistent slowness?)
z = (cyc - cyc.mean(axis=1, keepdims=True)) / cyc.std(axis=1, keepdims=True)
out["corr_consecutive"] = [float(np.mean(z[k] * z[k + 1])) for k in range(N - 1)]
out["corr_first_last"] = float(np.mean(z[0] * z[-1]))
m = cyc.mean(axis=0)
out["per_xcc_mean"] = {int(x): float(m[xcc == x].mean()) for x in np.unique(xcc)}
out["per_xcc_y0_range"] = {int(x): [int(y0[xcc == x].min()), int(y0[xcc == x].max())] for x in np.unique(xcc)}
out["per_ctile_mean_top5"] = sorted(((float(m[ct == c].mean()), int(c)) for c in np.unique(ct)), reverse=True)[:5]
out["edge_ctiles_mean"] = float(m[(ct == 0) | (ct == ct.max())].mean())
q = np.quantile(m, [0.5, 0.9, 0.99, 1.0])
out["wave_mean_quantiles"] = q.tolist()
slow = m > np.quantile(m, 0.98)
out["slowest_2pct"] = {"ctiles": np.unique(ct[slow]).tolist()[:40], "y0": np.unique(y0[slow]).tolist()[:40],
                       "xcc": np.bincount(xcc[slow], minlength=8).tolist()}
# what-if: the waves of a band pair (down band 2q over up band 2q-1, same
# column tile) share their rows at run time - each pair ends at 2 Td Tu / (Td + Tu)
ys = sorted(np.unique(y0[(ct > 0) & (ct < ct.max())]))
bidx = {y: k for k, y in enumerate(ys)}
sim = []
for l in range(N):
    tmax = 0.0
    byk = {}
    for w in range(cyc.shape[1]):
        if 0 < ct[w] < ct.max():
            byk[(int(ct[w]), bidx[int(y0[w])])] = cyc[l, w]
        else:
            tmax = max(tmax, cyc[l, w])
    for (c, b), t in byk.items():
        if b == 0:
            tmax = max(tmax, t)
        elif b % 2 == 0:
            tu = byk.get((c, b - 1))
            tmax = max(tmax, t if tu is None else 2 * t * tu / (t + tu))
        elif (c, b + 1) not in byk:
            tmax = max(tmax, t)
    sim.append(tmax)
out["pair_share_launch_max"] = sim
print(json.dumps(out, indent=1))
