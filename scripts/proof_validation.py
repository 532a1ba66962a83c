#!/usr/bin/env python3
"""Long-run check of the proof-mode convergence test: whole
cavity runs with the proof test and with exact residuals in every sweep
(CFD_PROOF=0) must give the same iteration count and residual at every step
and the same final fields, bit for bit. Each setting runs in a child process
(the switch is read at solver creation). Writes one JSON summary to stdout."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "computational-fluid-dynamics_amd"))

RUNS = [(256, 256, 300, 0), (500, 300, 100, 0), (1024, 1024, 6, 2000)]  # nx, ny, steps, cap (0: reference)

if len(sys.argv) == 1:
    out = []
    for nx, ny, steps, cap in RUNS:
        res = {}
        for proof in ("0", "1"):
            env = dict(os.environ, CFD_PROOF=proof, CFD_SMALL="0")
            r = subprocess.run([sys.executable, __file__, str(nx), str(ny), str(steps), str(cap)], env=env,
                               check=True, capture_output=True, text=True)
            res[proof] = json.loads(r.stdout.strip().splitlines()[-1])
        same = res["0"]["hist"] == res["1"]["hist"] and res["0"]["digest"] == res["1"]["digest"]
        out.append({"grid": f"{nx}x{ny}", "steps": steps, "cap": cap or None, "identical": same,
                    "converged_steps": sum(1 for k, _ in res["0"]["hist"] if k < (cap or 10000)),
                    "proof_fallbacks": res["1"]["fallbacks"], "s_exact": res["0"]["s"], "s_proof": res["1"]["s"]})
        print(json.dumps(out[-1]), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))
    sys.exit(0 if all(o["identical"] for o in out) else 1)

import hashlib  # noqa: E402

import cfd_amd as C  # noqa: E402

nx, ny, steps, cap = (int(a) for a in sys.argv[1:5])
cp = C.make_params("cavity", nx=nx, ny=ny, max_iters=cap or None)
s = C.solver_for(cp)
s.applyBoundaryConditions()
t0 = time.perf_counter()
hist = [list(s.step()) for _ in range(steps)]
el = time.perf_counter() - t0
h = hashlib.sha256()
for name in ("p", "u", "v"):
    h.update(s.field(name).tobytes())
tm = s.timing()
s.close()
print(json.dumps({"hist": hist, "digest": h.hexdigest(), "fallbacks": tm.proof_fallbacks, "s": round(el, 2)}))
