#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE per SOR launch (scripts/pmc_traffic.sh) -> HBM bytes
per launch with the gfx950 corrections (FETCH_SIZE x2 for 16-B/lane streaming
reads, WRITE_SIZE exact for 16-B/lane stores: MI355X_MICROARCH.md, HBM
[CDNA4]). CFD_COMMIT (the git commit of the profiled tree, set by the caller:
the GPU box has no .git) is recorded as "commit"; bench.py reports it as the
traffic's provenance, with the kernel's source hash. usage: pmc_traffic.py DIR KERNEL_SUBSTRING OUT.json [NX] [SWEEPS_PER_LAUNCH] [NY]"""
import csv
import glob
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "computational-fluid-dynamics_amd"))
from cfd_amd.provenance import source_hash  # noqa: E402

d, ksub, out = sys.argv[1], sys.argv[2], sys.argv[3]
nx = int(sys.argv[4]) if len(sys.argv) > 4 else 4096
sweeps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
ny = int(sys.argv[6]) if len(sys.argv) > 6 else nx


def per_dispatch(counter):
    f = glob.glob(f"{d}/{counter}/**/*counter_collection.csv", recursive=True)[0]
    v = {}
    for r in csv.DictReader(open(f)):
        if ksub in r["Kernel_Name"] and r["Counter_Name"] == counter:
            v[int(r["Dispatch_Id"])] = v.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    return v


fe, wr = per_dispatch("FETCH_SIZE"), per_dispatch("WRITE_SIZE")
# the middle half of the dispatches (steady state)
fv = sorted(fe.items())
wv = sorted(wr.items())
fv = [x for _, x in fv[len(fv) // 4: 3 * len(fv) // 4]]
wv = [x for _, x in wv[len(wv) // 4: 3 * len(wv) // 4]]
fetch_kib, write_kib = statistics.mean(fv), statistics.mean(wv)
rows = ny + 2
alg = 24.0 * rows * (nx + 2)
rd, wb = 2 * fetch_kib * 1024, write_kib * 1024
res = {"kernel_match": ksub, "nx": nx, "ny": ny, "rows": rows, "sweeps_per_launch": sweeps,
       "dispatches": [len(fv), len(wv)], "FETCH_SIZE_KiB_raw": fetch_kib, "WRITE_SIZE_KiB_raw": write_kib,
       "correction": "FETCH_SIZE x2 (gfx950 reports half of 16-B/lane streaming reads), WRITE_SIZE as is "
                     "(exact for 16-B/lane stores): MI355X_MICROARCH.md, HBM [CDNA4]",
       "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wb, "hbm_bytes_per_launch": rd + wb,
       "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": (rd + wb) / alg,
       "commit": os.environ.get("CFD_COMMIT") or None,
       # sha256 of the kernel's translation-unit sources on the profiled tree
       # (cfd_amd.provenance): bench.py drops the traffic when the sources changed
       "source_hash": source_hash(ksub),
       "command": f"scripts/pmc_traffic.sh (rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE, separate passes), {d}"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
