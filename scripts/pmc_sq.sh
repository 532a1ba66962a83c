#!/usr/bin/env bash
# SQ stall-class counters of one SOR kernel per workload (one rocprofv3 --pmc
# pass each, middle half of the launches): WAVE_CYCLES = WAIT_ANY (parked at
# s_waitcnt / barrier) + WAIT_INST_ANY (issue stalls) + ACTIVE_INST_ANY, in
# quad-cycles; GRBM_GUI_ACTIVE gives the clock (cycles per launch).
# WORKLOADS="name:kernel-substring:bench args;..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=${OUT:-gpurun_out/pmc_sq}; mkdir -p $D
CTR=${CTR:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE}
IFS=';' read -ra WL <<< "$WORKLOADS"
for w in "${WL[@]}"; do
  n=${w%%:*}; rest=${w#*:}; kn=${rest%%:*}; a=${rest#*:}
  timeout -s KILL 120 rocprofv3 --pmc $CTR -d $D/$n -o run --output-format csv -- python3 bench.py --no-cpu-baseline --lex-steps 0 --steps 1 --warmup 0 --max-iters 400 $a > $D/$n.out 2>&1 || exit 1
  f=$(find $D/$n -name '*counter_collection.csv' | head -1)
  python3 - "$f" "$kn" "$n" <<'PY'
import csv, sys, collections, json
v = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Kernel_Name"]:
        v[r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, x in sorted(v.items()):
    x = sorted(x)[len(x) // 4: 3 * len(x) // 4] or x
    out[k] = sum(x) / len(x)
print(json.dumps({"workload": sys.argv[3], "kernel": sys.argv[2], "per_launch": out}))
PY
done
