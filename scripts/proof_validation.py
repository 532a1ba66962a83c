#!/usr/bin/env python3
"""Long-run check of the proof-mode convergence test: whole
cavity runs with the proof test and with exact residuals in every sweep
(proof_test="off") must give the same iteration count and residual at every
step and the same final fields, bit for bit. Writes one JSON summary to stdout."""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "computational-fluid-dynamics_amd"))

import cfd_amd as C  # noqa: E402

RUNS = [(256, 256, 300, 0), (500, 300, 100, 0), (1024, 1024, 6, 2000)]  # nx, ny, steps, cap (0: reference)


def run(nx, ny, steps, cap, proof):
    cp = C.make_params("cavity", nx=nx, ny=ny, max_iters=cap or None)
    s = C.solver_for(cp, ordering="rb", small_solve="off", proof_test=proof)
    s.applyBoundaryConditions()
    t0 = time.perf_counter()
    hist = [list(s.step()) for _ in range(steps)]
    el = time.perf_counter() - t0
    h = hashlib.sha256()
    for name in ("p", "u", "v"):
        h.update(s.field(name).tobytes())
    tm = s.timing()
    s.close()
    return {"hist": hist, "digest": h.hexdigest(), "fallbacks": tm.proof_fallbacks, "s": round(el, 2)}


out = []
for nx, ny, steps, cap in RUNS:
    res = {p: run(nx, ny, steps, cap, p) for p in ("off", "on")}
    same = res["off"]["hist"] == res["on"]["hist"] and res["off"]["digest"] == res["on"]["digest"]
    out.append({"grid": f"{nx}x{ny}", "steps": steps, "cap": cap or None, "identical": same,
                "converged_steps": sum(1 for k, _ in res["off"]["hist"] if k < (cap or 10000)),
                "proof_fallbacks": res["on"]["fallbacks"], "s_exact": res["off"]["s"], "s_proof": res["on"]["s"]})
    print(json.dumps(out[-1]), file=sys.stderr, flush=True)
print(json.dumps(out, indent=1))
sys.exit(0 if all(o["identical"] for o in out) else 1)
