"""Resident solve vs LDS tiles: iteration counts, fallbacks, launches, solve time (GPU)."""
import sys
sys.path.insert(0, "computational-fluid-dynamics_amd"); sys.path.insert(0, "oracle")
import numpy as np
import cfd_amd as C
from cfd_amd import _lib
for nx, ny, cap in [(300, 200, 600), (1024, 64, 600), (1024, 1024, 200), (1024, 1024, 10000)]:
    cp = C.make_params("cavity", nx=nx, ny=ny, max_iters=cap)
    for res in (1, 0):
        g = C.CavitySolver(cp, ordering="rb", device=0, small_solve="off", tuning={"resident": res, "tile_rounds": 1})
        g.applyBoundaryConditions()
        h = [g.step()]
        g.reset_timing()
        h += [g.step() for _ in range(2)]
        tm = g.timing()
        p = g.field("p").copy()
        print(nx, ny, cap, "res" if res else "tile", h, "fallbacks", tm.proof_fallbacks, "launches", tm.poisson_launches,
              "ms/solve", round(tm.poisson_ms / 2, 3), "us/sweep", round(1000 * tm.poisson_ms / 2 / cap, 3),
              _lib.SOR_KERNEL[tm.sor_kernel], "psum", float(np.abs(p).sum()), flush=True)
        g.close()
