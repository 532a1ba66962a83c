"""Resident reference-order solve vs the lexw march: iteration counts, fallbacks, solve time (GPU)."""
import sys
sys.path.insert(0, "computational-fluid-dynamics_amd"); sys.path.insert(0, "oracle")
import numpy as np
import cfd_amd as C
from cfd_amd import _lib
for nx, ny, cap in [(1024, 64, 600), (1024, 1024, 2000), (1024, 1024, 10000)]:
    cp = C.make_params("cavity", nx=nx, ny=ny, max_iters=cap)
    for res in (1, 0):
        g = C.CavitySolver(cp, ordering="lex", device=0, small_solve="off", tuning={"resident": res})
        g.applyBoundaryConditions()
        h = [g.step()]
        g.reset_timing()
        h += [g.step() for _ in range(2)]
        tm = g.timing()
        p = g.field("p").copy()
        print(nx, ny, cap, "res" if res else "lexw", h, "fallbacks", tm.proof_fallbacks, "launches", tm.poisson_launches,
              "ms/solve", round(tm.poisson_ms / 2, 3), "GLUPS", round(nx * ny * cap / (tm.poisson_ms / 2) / 1e6, 1),
              _lib.SOR_KERNEL[tm.sor_kernel], "psum", float(np.abs(p).sum()), flush=True)
        g.close()
