#!/usr/bin/env python3
"""Time the reference-order sequential source sum (seqsum.hip) at the BASELINE
open-case sizes: buildSourceTerm() in ordering="lex" (source pass + the
sequential sum + mean removal), against the same call in red-black order
(tree sum). Writes JSON to stdout."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "computational-fluid-dynamics_amd"))

import torch  # noqa: E402,F401  (HIP runtime first)

import cfd_amd as C  # noqa: E402

out = []
for case, nx, ny in (("channel", 4096, 512), ("backwards_step", 8192, 512)):
    r = {"case": case, "grid": f"{nx}x{ny}", "terms": nx * ny}
    for ordering in ("lex", "rb"):
        s = C.solver_for(C.make_params(case, nx=nx, ny=ny, re=1000.0 if case == "channel" else 400.0),
                         ordering=ordering)
        s.computeTentativeVelocities()
        s.buildSourceTerm()
        s.synchronize()
        n = 3
        t0 = time.perf_counter()
        for _ in range(n):
            s.buildSourceTerm()
        s.synchronize()
        r[f"{ordering}_ms"] = round((time.perf_counter() - t0) / n * 1e3, 3)
        s.close()
    r["lex_ns_per_term"] = round((r["lex_ms"] - r["rb_ms"]) * 1e6 / r["terms"], 3)
    out.append(r)
    print(json.dumps(r), file=sys.stderr, flush=True)
print(json.dumps(out, indent=1))
