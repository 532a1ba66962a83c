#!/usr/bin/env python3
"""Sweep SOR-kernel launch knobs on the bench grid (4096^2 cavity): each config
gets a fresh solver (knobs are read at construction) and times N fixed
sweeps with HIP events on the solver's stream. Prints one line per config."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "computational-fluid-dynamics_amd"))
import cfd_amd as C  # noqa: E402

N = int(os.environ.get("SWEEP_ITERS", "300"))
nx = int(os.environ.get("SWEEP_NX", "4096"))
case = os.environ.get("SWEEP_CASE", "cavity")
configs = [c.split(",") for c in sys.argv[1:]] or [["wave", "", "3", ""]]
for variant, bpc, flags, minth in configs:
    # bpc: blocks per CU (block march) or waves per SIMD (wave march)
    for k, v in (("CFD_POISSON_KERNEL", variant), ("CFD_MARCH_BLOCKS_PER_CU", bpc if variant == "march" else ""),
                 ("CFD_WAVE_WPS", bpc if variant == "wave" else ""), ("CFD_MARCH_FLAGS", flags),
                 ("CFD_MARCH_MIN_TH", minth)):
        if v:
            os.environ[k] = v
        else:
            os.environ.pop(k, None)
    cp = C.make_params(case, nx=nx, ny=nx, max_iters=N)
    s = C.solver_for(cp)
    if case == "cavity":
        s.applyBoundaryConditions()
    s.computeTentativeVelocities()
    if case != "cavity":
        s.applyTentativeBoundaryConditions()
    s.buildSourceTerm()
    s.solverPressurePoisson()  # warm
    s.reset_timing()
    t0 = time.perf_counter()
    it, _ = s.solverPressurePoisson()
    el = time.perf_counter() - t0
    tm = s.timing()
    us = tm.poisson_ms * 1e3 / max(tm.poisson_launches, 1)
    gbs = 24.0 * (nx + 2) * (nx + 2) / (us * 1e-6) / 1e9
    print(f"{variant:6s} bpc={bpc or 'auto':4s} flags={flags or '3':2s} minth={minth or '24':3s}  {us:8.2f} us/sweep"
          f"  {gbs:7.1f} GB/s  iters={it} wall={el:.2f}s", flush=True)
    s.close()
