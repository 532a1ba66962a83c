#!/usr/bin/env python3
"""Durations of the lexw SOR launches along one solve, from a rocprofv3 kernel
trace (scripts/prof_lex.sh): mean / min / max per block of launches, gaps."""
import csv
import statistics
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/proflex/run_kernel_trace.csv"
rows = [r for r in csv.DictReader(open(path)) if "lexw" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows]
kind = ["S" if "false" in r["Kernel_Name"] else "R" for r in rows]
n = len(d) // 2  # second of two solves (the first is the warmup step)
seg, ks = d[n:], kind[n:]
blk = int(sys.argv[2]) if len(sys.argv) > 2 else 250
print("launches per solve", len(seg))
for a in range(0, len(seg), blk):
    c = seg[a:a + blk]
    print(f"{a:6d} {ks[a]} mean {statistics.mean(c):7.1f} min {min(c):7.1f} max {max(c):7.1f} us")
t = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows[n:]]
print("ramp ms", sum(x for x, k in zip(seg, ks) if k == "R") / 1000, "steady ms",
      sum(x for x, k in zip(seg, ks) if k == "S") / 1000, "span ms", (t[-1][1] - t[0][0]) / 1e6)
