#!/usr/bin/env bash
# SQ counters of the one-workgroup reference-order solve (smlex.hip) on the
# reference's own cases: two rocprofv3 --pmc passes per case, per-launch
# averages (python scripts/smlex_run.py drives N steps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=${OUT:-gpurun_out/prof_smlex}; mkdir -p $D
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM"
for c in ${CASES:-cavity channel backwards_step}; do
  n=20; [ $c = backwards_step ] && n=4
  k=1
  for ctr in "$P1" "$P2"; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr -d $D/${c}_$k -o run --output-format csv -- python3 scripts/smlex_run.py $c $n > $D/${c}_$k.out 2>&1 || exit 1
    f=$(find $D/${c}_$k -name '*counter_collection.csv' | head -1)
    python3 - "$f" "$c" "$k" <<'PY'
import csv, sys, collections, json
v = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "smlex" in r["Kernel_Name"]:
        v[r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: sum(x) / len(x) for k, x in sorted(v.items())}
print(json.dumps({"case": sys.argv[2], "pass": int(sys.argv[3]), "launches": len(next(iter(v.values()), [])), "per_launch": out}))
PY
    k=$((k+1))
  done
done
