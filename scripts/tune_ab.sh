#!/usr/bin/env bash
# Launch-plan knobs of the headline cavity launch (bench lines, same build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${OUT:-gpurun_out/tune_ab}; mkdir -p $D
A="--no-cpu-baseline --lex-steps 0 --steps 3 --warmup 1 ${ARGS:-}"
for t in ${TUNES:-none pair_wps=1 pair_wps=3 pair_edge_pct=60 pair_edge_pct=100 march_min_th=48 march_min_th=96}; do
  extra=""; [ "$t" != none ] && extra="--tune $t"
  timeout -k 10 200 python3 -u bench.py $A $extra > $D/$t.json 2> $D/$t.err || { tail -3 $D/$t.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$D/$t.json')); r=d['roofline']
print('$t', d['value'], 'MLUPS', r['avg_launch_us'], 'us/launch frac', r['frac'])"
done
