"""Debug helper: per-step (iterations, residual) of the reference cavity with
1, 2 and 3 sweeps per launch."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "computational-fluid-dynamics_amd"))
import numpy as np
import cfd_amd as C

cp = C.reference_defaults("cavity")
gs = {spl: C.CavitySolver(cp, device=0, sweeps_per_launch=spl) for spl in (1, 2, 3)}
for step in range(6):
    r = {spl: g.step() for spl, g in gs.items()}
    p = {spl: g.field("p") for spl, g in gs.items()}
    for spl in (2, 3):
        print(step, spl, r[spl], r[1], r[spl] == r[1], np.array_equal(p[spl].view(np.int64), p[1].view(np.int64)))
