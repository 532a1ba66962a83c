"""Dump the open cases' raw source terms (before the mean removal) at the
bench configurations after a few reference-order steps, for studying the
sequential source sum's running partial sums (scripts/dbg/seqsum_study.py).
GPU box: python scripts/dbg/dump_src.py -> gpurun_out/src_<case>.npz with
f<step> = the (ny, nx) interior terms as source_kernel forms them (numpy, the
same operations, no contraction) and mean<step> = the mean the library took
(src + mean == f up to the subtraction's rounding)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "computational-fluid-dynamics_amd"))
import cfd_amd as C  # noqa: E402

CASES = {"channel": dict(nx=4096, ny=512, re=1000), "backwards_step": dict(nx=8192, ny=512, re=400)}
STEPS = [int(s) for s in os.environ.get("DUMP_STEPS", "20").split(",")]
os.makedirs("gpurun_out", exist_ok=True)
for case, kw in CASES.items():
    cp = C.make_params(case, **kw)
    g = {"channel": C.ChannelSolver, "backwards_step": C.BackwardsStepSolver}[case](cp, ordering="lex")
    out = {}
    done = 0
    for s in STEPS:
        g.run_steps(s - done)
        done = s
        # one more step's first stages (the fields they write are rebuilt by
        # the next step from u, v; the dump ends the run anyway)
        g.applyBoundaryConditions()
        g.computeTentativeVelocities()
        g.applyTentativeBoundaryConditions()
        us, vs = g.field("us"), g.field("vs")
        ny, nx = cp.ny, cp.nx
        du = us[1:ny + 1, 1:nx + 1] - us[1:ny + 1, 0:nx]
        dv = vs[1:ny + 1, 1:nx + 1] - vs[0:ny, 1:nx + 1]
        f = (cp.rho / cp.dt) * (du * (1.0 / cp.dx) + dv * (1.0 / cp.dy))
        g.buildSourceTerm()
        src = g.field("src")[1:ny + 1, 1:nx + 1]
        fl = src != 0.0
        out[f"f{s}"] = f
        out[f"mean{s}"] = np.median((f - src)[fl])
        print(case, s, "f range", np.abs(f).max(), "mean est", np.median((f - src)[fl]), flush=True)
    np.savez_compressed(f"gpurun_out/src_{case}.npz", **out)
