#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the reference itself.

The reference solvers (/root/reference/{cavity-01,channel-01,backwards_step-01}.cpp)
are compiled by oracle/build_ref.sh into oracle/_ref/ and run there, in
oracle/_ref/runs/<case>/ (their hard-coded configurations; they take no CLI).
This script then extracts DATA only — VTK field values of selected frames and the
stdout/stderr residual-log lines — into:

  tests/golden/ref_fields.npz   float64 arrays "<case>/<frame>/<field>", shape (ny, nx)
  tests/golden/ref_logs.json    {"<case>": {"header": [...], "steps": [...], "warnings": [...],
                                 "vtk_sha256": {"<frame>": hex digest of the reference's frame file}}}

The VTK writer prints fixed-point with 6 decimals (cavity-01.cpp:110 sets
std::fixed/setprecision(6) on the file stream), so each stored value is the
exact double nearest to the printed decimal; '%.6f' of it reproduces the text.

The backwards-step case hits the 10000-iteration SOR cap on nearly every step
(about 1 s per step on one core), so only its early frames are kept: the run is
stopped once frame STEP_LAST_FRAME has been written.

Run from the repo root:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF_DIR = os.environ.get("CFD_REFERENCE_DIR", "/root/reference")
REF_BIN = os.path.join(ROOT, "oracle", "_ref")
RUNS = os.path.join(REF_BIN, "runs")
OUT = os.path.dirname(os.path.abspath(__file__))

CASES = {
    # case: (binary, vtk base name, frames kept)
    "cavity": ("cavity", "cavity_flow", [100, 200, 2520]),
    "channel": ("channel", "channel_flow", [100, 200, 1537]),
    "backwards_step": ("backwards_step", "backwards_step", [10, 20]),
}
STEP_LAST_FRAME = 20
FIELDS = ("u_velocity", "v_velocity", "pressure", "vorticity")
ANSI = re.compile(r"\x1b\[[0-9;]*m")


def run_reference(case: str) -> str:
    binary, base, frames = CASES[case]
    wd = os.path.join(RUNS, case)
    done = os.path.join(wd, "DONE")
    last = os.path.join(wd, "vtk_output", f"{base}_{frames[-1]:06d}.vtk")
    if os.path.exists(done) or (case == "backwards_step" and os.path.exists(last)):
        return wd
    os.makedirs(wd, exist_ok=True)
    with open(os.path.join(wd, "stdout.txt"), "w") as so, open(os.path.join(wd, "stderr.txt"), "w") as se:
        proc = subprocess.Popen([os.path.join(REF_BIN, binary)], cwd=wd, stdout=so, stderr=se)
        if case == "backwards_step":
            nxt = os.path.join(wd, "vtk_output", f"{base}_{STEP_LAST_FRAME + 10:06d}.vtk")
            while proc.poll() is None and not os.path.exists(nxt):
                time.sleep(1.0)
            if proc.poll() is None:
                proc.terminate()
                proc.wait()
        else:
            proc.wait()
            with open(done, "w") as f:
                f.write(str(proc.returncode))
    return wd


def parse_vtk(path: str) -> dict[str, np.ndarray]:
    with open(path) as f:
        lines = f.read().split("\n")
    dims = next(l for l in lines if l.startswith("DIMENSIONS")).split()
    nx, ny = int(dims[1]), int(dims[2])
    out = {}
    k = 0
    while k < len(lines):
        parts = lines[k].split()
        if len(parts) >= 2 and parts[0] == "SCALARS" and parts[1] in FIELDS:
            vals = np.array([float(x) for x in lines[k + 2 : k + 2 + nx * ny]], dtype=np.float64)
            out[parts[1]] = vals.reshape(ny, nx)
            k += 2 + nx * ny
        else:
            k += 1
    return out


def parse_logs(wd: str) -> dict:
    with open(os.path.join(wd, "stdout.txt")) as f:
        out = [ANSI.sub("", l.rstrip("\n")) for l in f]
    with open(os.path.join(wd, "stderr.txt")) as f:
        err = [ANSI.sub("", l.rstrip("\n")) for l in f]
    return {
        "header": [l for l in out if l.startswith(("Grid:", "Time:", "Reynolds=", "Relaxation", "Geometry setup"))],
        "steps": [l for l in out if l.startswith("Step ")],
        "warnings": [l for l in err if "Warning" in l],
    }


def main() -> int:
    if not os.path.isdir(REF_DIR):
        print(f"reference tree {REF_DIR} absent; fixtures are committed, nothing to do")
        return 0
    subprocess.check_call([os.path.join(ROOT, "oracle", "build_ref.sh"), REF_DIR])
    arrays = {}
    logs = {}
    for case, (_, base, frames) in CASES.items():
        wd = run_reference(case)
        for fr in frames:
            fields = parse_vtk(os.path.join(wd, "vtk_output", f"{base}_{fr:06d}.vtk"))
            for name, a in fields.items():
                arrays[f"{case}/{fr}/{name}"] = a
        lg = parse_logs(wd)
        lg["vtk_sha256"] = {}
        for fr in [0] + frames:
            with open(os.path.join(wd, "vtk_output", f"{base}_{fr:06d}.vtk"), "rb") as fh:
                lg["vtk_sha256"][str(fr)] = hashlib.sha256(fh.read()).hexdigest()
        if case == "backwards_step":
            lg["steps"] = [l for l in lg["steps"] if int(l.split()[1].split("/")[0]) <= STEP_LAST_FRAME]
            # one warning per capped step, in step order; keep a prefix long
            # enough to cover the kept steps (tests compare prefixes)
            lg["warnings"] = lg["warnings"][: 2 * STEP_LAST_FRAME]
        logs[case] = lg
    np.savez_compressed(os.path.join(OUT, "ref_fields.npz"), **arrays)
    with open(os.path.join(OUT, "ref_logs.json"), "w") as f:
        json.dump(logs, f, indent=1)
    print(f"wrote {len(arrays)} arrays and logs for {list(logs)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
