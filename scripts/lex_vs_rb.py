#!/usr/bin/env python3
"""Red-black vs the reference's lexicographic SOR ordering at BASELINE sizes (CPU oracle).

The reference's SOR sweep (cavity-01.cpp:635-678) is lexicographic; the GPU's
fast path is red-black (bit-exact against oracle/ ORC_RB). Where the solve
converges to its tolerance the two orderings reach the same fixed point; where
the 10000-sweep cap is hit they stop at different iterates. This script
measures the gap on the north-star metric (centerline u/v relative L2) after
whole timesteps of the cavity.

  python scripts/lex_vs_rb.py run N ORDER STEPS OUT.npz   (ORDER: lex | rb)
  python scripts/lex_vs_rb.py compare LEX.npz RB.npz OUT.json

`run` is single-threaded (the oracle's C loop); 4096² takes ~20 min per
ordering per step at the 10000-sweep cap.
"""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "computational-fluid-dynamics_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402


def centerlines(uc, vc, nx, ny):
    ic = (nx + 1) // 2
    jc = (ny + 1) // 2
    return uc[1:ny + 1, ic].copy(), vc[jc, 1:nx + 1].copy()


def run(n: int, order: str, steps: int, out: str) -> None:
    import oracle as O
    from cfd_amd.params import make_params

    cp = make_params("cavity", re=1000.0, nx=n, ny=n, max_iters=10000)
    o = O.Oracle(cp, ordering=O.LEX if order == "lex" else O.RB)
    its, ress, secs = [], [], []
    for _ in range(steps):
        t0 = time.perf_counter()
        it, res = o.step()
        secs.append(time.perf_counter() - t0)
        its.append(it)
        ress.append(res)
        print(f"{order} {n}: step {len(its)} iterations {it} residual {res:.6e} ({secs[-1]:.1f} s)", flush=True)
    o.centers()
    u, v = centerlines(o.field("uc"), o.field("vc"), n, n)
    p = o.field("p")
    np.savez(out, u=u, v=v, p_center=p[(n + 1) // 2, :].copy(), p_vcenter=p[:, (n + 1) // 2].copy(),
             its=np.array(its), res=np.array(ress), secs=np.array(secs), n=n, tol_factor=cp.tol_factor)


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def compare(lex: str, rb: str, out: str) -> None:
    L, R = np.load(lex), np.load(rb)
    scale = np.linalg.norm(L["u"])
    d = {
        "n": int(L["n"]),
        "workload": f"lid-driven cavity Re=1000, {int(L['n'])}^2, dt from the reference CFL rule, "
                    "SOR tolerance 1e-9*max|src|, cap 10000 sweeps/step",
        "steps": int(len(L["its"])),
        "sor_iterations_lex": [int(x) for x in L["its"]],
        "sor_iterations_rb": [int(x) for x in R["its"]],
        "final_residual_lex": [float(x) for x in L["res"]],
        "final_residual_rb": [float(x) for x in R["res"]],
        "centerline_u_rel_l2": rel_l2(R["u"], L["u"]),
        "centerline_v_rel_l2": float(np.linalg.norm(R["v"] - L["v"]) / max(scale, np.linalg.norm(L["v"]))),
        "centerline_p_rel_l2": rel_l2(R["p_center"], L["p_center"]),
        "cpu_seconds_per_step_lex": [float(x) for x in L["secs"]],
        "cpu_seconds_per_step_rb": [float(x) for x in R["secs"]],
        "bar": 1e-6,
        "how": "oracle/ (gcc -O2, single core): ORC_LEX = the reference's sweep order (pinned to the reference "
               "binaries by tests/test_oracle_golden.py), ORC_RB = the GPU path's order (bit-exact vs the HIP "
               "kernels); scripts/lex_vs_rb.py",
    }
    with open(out, "w") as fh:
        json.dump(d, fh, indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), sys.argv[5])
    else:
        compare(sys.argv[2], sys.argv[3], sys.argv[4])
