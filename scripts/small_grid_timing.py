#!/usr/bin/env python3
"""Reference-sized runs on the GPU (one-workgroup LDS solve, small.hpp) vs the
reference's loop restated in C (oracle, lexicographic order, one core): the
reference's default cavity run (63², cavity-01.cpp:311-318, run() loop) and
the channel / step defaults, N steps each. Writes JSON to stdout."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "computational-fluid-dynamics_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import torch  # noqa: E402,F401  (HIP runtime first)

import cfd_amd as C  # noqa: E402
import oracle as O  # noqa: E402


def run(case, steps, cpu_steps):
    cp = C.reference_defaults(case)
    g = C.solver_for(cp)
    if case == "cavity":
        g.applyBoundaryConditions()
    g.step()
    g.synchronize()
    t0 = time.perf_counter()
    its = [g.step()[0] for _ in range(steps)]
    g.synchronize()
    gpu_s = time.perf_counter() - t0
    tm = g.timing()
    g.close()
    o = O.Oracle(cp, ordering=O.LEX)
    if case != "cavity":
        o.velocity_bc(False)
    o.step()
    t0 = time.perf_counter()
    cits = [o.step()[0] for _ in range(cpu_steps)]
    cpu_s = time.perf_counter() - t0
    cpu_per_step = cpu_s / cpu_steps
    return {"case": case, "grid": f"{cp.nx}x{cp.ny}", "steps": steps,
            "gpu_s": round(gpu_s, 4), "gpu_ms_per_step": round(gpu_s / steps * 1e3, 4),
            "gpu_sor_iters_per_step": round(sum(its) / steps, 1),
            "gpu_solve_launches": tm.poisson_launches,
            "cpu_steps": cpu_steps, "cpu_ms_per_step": round(cpu_per_step * 1e3, 4),
            "cpu_sor_iters_per_step": round(sum(cits) / cpu_steps, 1),
            "cpu_kind": "oracle lexicographic loop (the reference's order), gcc -O2, 1 core",
            "speedup_per_step": round(cpu_per_step / (gpu_s / steps), 2)}


if __name__ == "__main__":
    out = []
    for case, n, ncpu in (("cavity", 2519, 300), ("channel", 100, 20), ("backwards_step", 50, 10)):
        out.append(run(case, n, ncpu))
        print(json.dumps(out[-1]), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))
