#!/usr/bin/env bash
# SQ counters of the resident solve at 1024^2 (rocprofv3 --pmc, two passes):
# one warm-up step (falls back: step 1's first iteration is left open), one
# resident step; the resident launch with the most waves-cycles is reported.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=${OUT:-gpurun_out/pmc_res}; mkdir -p $D
A="--no-cpu-baseline --lex-steps 0 --steps 1 --warmup 1 --max-iters 2000 --nx ${NX:-1024} --ny ${NY:-1024} --tune resident=1"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
i=0
for ctr in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d $D/p$i -o run --output-format csv -- python3 bench.py $A > $D/p$i.out 2>&1 || exit 1
done
python3 - $D <<'PY'
import csv, sys, glob, collections, json
d = sys.argv[1]
out = {}
for f in glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if "poisson_resident" in r["Kernel_Name"]:
            per[r.get("Dispatch_Id", r.get("Correlation_Id"))][r["Counter_Name"]] = float(r["Counter_Value"])
    best = max(per.values(), key=lambda x: x.get("GRBM_GUI_ACTIVE", 0))
    out.update(best)
print(json.dumps(out, indent=1))
PY
