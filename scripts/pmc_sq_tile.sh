#!/usr/bin/env bash
# SQ counters of the LDS-tile SOR kernel (cavity 1024^2, channel 4096x512): one pass each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/pmc_sq_tile; mkdir -p $D
for w in "cav1k:--case cavity --nx 1024 --ny 1024" "ch:--case channel --nx 4096 --ny 512"; do
  n=${w%%:*}; a=${w#*:}
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM -d $D/$n -o run --output-format csv -- python3 bench.py --no-cpu-baseline --lex-steps 0 --steps 1 --warmup 0 --max-iters 400 $a > $D/$n.out 2>&1 || exit 1
  f=$(find $D/$n -name '*counter_collection.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
v = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "poisson_tile_kernel" in r["Kernel_Name"]:
        v[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, x in sorted(v.items()):
    x = sorted(x)[len(x) // 4: 3 * len(x) // 4] or x
    print(f"  {k}: {sum(x) / len(x):.4g} per launch ({len(x)} launches)")
PY
done
