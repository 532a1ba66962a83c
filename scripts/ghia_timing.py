#!/usr/bin/env python3
"""ms per cavity step (Re=100) at reference-like sizes: the one-workgroup solve
(small.hpp) against the multi-launch solve (small_solve="off"), for choosing
the crossover (Solver::use_small)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "computational-fluid-dynamics_amd"))

import cfd_amd as C  # noqa: E402

for small in ("on", "off"):
    for n, dt in ((63, 0.0), (96, 0.0), (128, 1e-3)):
        cp = C.make_params("cavity", re=100.0, nx=n, ny=n, dt=dt if dt > 0 else None)
        s = C.solver_for(cp, ordering="rb", small_solve=small)
        s.applyBoundaryConditions()
        s.step()
        t0 = time.perf_counter()
        its = [s.step()[0] for _ in range(200)]
        el = time.perf_counter() - t0
        print(f"small_solve={small} {n}^2 dt={cp.dt:g}: {el / 200 * 1e3:.3f} ms/step, "
              f"{sum(its) / len(its):.0f} iterations/step", flush=True)
        s.close()
