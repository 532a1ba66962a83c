#!/usr/bin/env python3
"""Mean SQ counters of the lexw launches in a window of dispatches (steady
phase by default) from a rocprofv3 counter_collection.csv."""
import collections
import csv
import sys

path = sys.argv[1]
kind = sys.argv[2] if len(sys.argv) > 2 else "false"  # steady kernel
d = collections.OrderedDict()
for r in csv.DictReader(open(path)):
    if (sys.argv[3] if len(sys.argv) > 3 else "lexw") not in r["Kernel_Name"]:
        continue
    e = d.setdefault(r["Dispatch_Id"], {"k": "false" if "false>" in r["Kernel_Name"] else "true",
                                        "vgpr": r["VGPR_Count"], "sgpr": r["SGPR_Count"]})
    e[r["Counter_Name"]] = float(r["Counter_Value"])
sel = [e for e in d.values() if e["k"] == kind]
sel = sel[len(sel) // 4: 3 * len(sel) // 4] or sel
agg = collections.Counter()
for e in sel:
    for k, v in e.items():
        if k.startswith(("SQ_", "TCC_", "TCP_", "TA_", "GRBM_")):
            agg[k] += v / len(sel)
print(f"{len(sel)} dispatches of kernel<.., {kind}>  vgpr {sel[0]['vgpr']} sgpr {sel[0]['sgpr']}")
for k, v in sorted(agg.items()):
    print(f"  {k:24s} {v:16.0f}")
if "SQ_INSTS_VALU" in agg and "SQ_WAVES" in agg:
    print("  VALU per wave", agg["SQ_INSTS_VALU"] / agg["SQ_WAVES"], " SALU per wave", agg.get("SQ_INSTS_SALU", 0) / agg["SQ_WAVES"])
