#!/usr/bin/env python3
"""Reference-order launch shape at the BASELINE sizes: ms per capped solve for
tiles per launch (CFD_TUNE_LEXW_WAVES) and, for the cavity, 4 vs 5 sweeps per
launch. One JSON line per setting (performance only: every setting gives the
same bits, tests/test_gpu_lexw.py)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "computational-fluid-dynamics_amd"))
import torch  # noqa: E402,F401  (one HIP runtime: torch first)

import cfd_amd as C  # noqa: E402

K = int(os.environ.get("ITERS", "3000"))
CASES = [("channel", dict(re=1000.0, nx=4096, ny=512), [0]), ("backwards_step", dict(re=400.0, nx=8192, ny=512), [0]),
         ("cavity", dict(re=1000.0, nx=4096, ny=4096), [4, 5])]
for case, kw, spls in CASES:
    if os.environ.get("CASES") and case not in os.environ["CASES"].split(","):
        continue
    cp = C.make_params(case, max_iters=K, **kw)
    for spl in spls:
        for waves, rpct in [tuple(int(v) for v in w.split(":")) for w in
                            os.environ.get("WAVES", "0:0,256:0,512:0,1024:0,1536:0,0:50,0:75,0:100").split(",")]:
            s = C.solver_for(cp, ordering="lex", sweeps_per_launch=spl)
            if waves:
                s.set_tuning("lexw_waves", waves)
            s.set_tuning("lexw_ramp_pct", rpct)
            if case == "cavity":
                s.applyBoundaryConditions()
            s.step()
            s.synchronize()
            s.reset_timing()
            t0 = time.perf_counter()
            it, res = s.step()
            s.synchronize()
            el = time.perf_counter() - t0
            tm = s.timing()
            s.close()
            print(json.dumps({"case": case, "spl": spl, "lexw_waves": waves or "auto", "ramp_pct": rpct, "iters": it,
                              "ms_step": round(el * 1e3, 2), "poisson_ms": round(tm.poisson_ms, 2),
                              "launches": tm.poisson_launches,
                              "steady_us": round(tm.poisson_steady_ms / max(tm.poisson_steady_launches, 1) * 1e3, 2),
                              "steady_launches": tm.poisson_steady_launches,
                              "us_per_sweep": round(tm.poisson_ms / max(it, 1) * 1e3, 3)}), flush=True)
