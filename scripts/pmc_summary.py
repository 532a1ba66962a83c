#!/usr/bin/env python3
"""HBM traffic per launch of the SOR kernel from the two rocprofv3 PMC passes
written by scripts/profile_round.sh (FETCH_SIZE and WRITE_SIZE, one pass each).

Corrections (MI355X_MICROARCH.md, section "HBM [CDNA4]"): on gfx950 FETCH_SIZE
reports exactly half of the bytes of a 16-B-per-lane streaming read, so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores. Counter units
are KiB per dispatch (summed over the XCDs by rocprofv3).

usage: pmc_summary.py <pmc_dir> <kernel-substring> <out.json> [sweeps_per_launch]
"""
from __future__ import annotations

import csv
import json
import os
import sys

NX = 4096
ROWS = 4098  # 4096 interior rows + 2 ghost rows (one strip)


def mean_counter(path: str, kernel: str, counter: str) -> tuple[float, int]:
    vals = []
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} samples for {kernel!r} in {path}")
    return sum(vals) / len(vals), len(vals)


def main() -> None:
    d, kernel, out = sys.argv[1], sys.argv[2], sys.argv[3]
    spl = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    f_kib, nf = mean_counter(os.path.join(d, "FETCH_SIZE", "run_counter_collection.csv"), kernel, "FETCH_SIZE")
    w_kib, nw = mean_counter(os.path.join(d, "WRITE_SIZE", "run_counter_collection.csv"), kernel, "WRITE_SIZE")
    rd = 2.0 * f_kib * 1024.0
    wr = w_kib * 1024.0
    algo = 24 * ROWS * (NX + 2)
    res = {
        "kernel": kernel,
        "nx": NX,
        "rows": ROWS,
        "sweeps_per_launch": spl,
        "dispatches": [nf, nw],
        "FETCH_SIZE_KiB_raw": f_kib,
        "WRITE_SIZE_KiB_raw": w_kib,
        "correction": "FETCH_SIZE x2 (gfx950 reports half of 16-B/lane streaming reads), WRITE_SIZE as is "
                      "(exact for 16-B/lane stores): MI355X_MICROARCH.md, HBM [CDNA4]",
        "hbm_read_bytes_per_launch": rd,
        "hbm_write_bytes_per_launch": wr,
        "hbm_bytes_per_launch": rd + wr,
        "algorithmic_bytes_per_launch": algo,
        "traffic_over_algorithmic": (rd + wr) / algo,
        "command": "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE (separate passes) -- python3 bench.py --steps 1 "
                   "--warmup 0 --max-iters 100 --no-cpu-baseline",
    }
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
