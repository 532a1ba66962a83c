#!/usr/bin/env bash
# Launch-plan knobs of the open cases' proof-mode march launches (bench lines only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${OUT:-gpurun_out/open_tune}
mkdir -p $D
A="--no-cpu-baseline --lex-steps 0 --steps 1 --warmup 1 --tile-rounds 0"
for c in "channel --nx 4096 --ny 512" "backwards_step --nx 8192 --ny 512 --re 400"; do
  for t in "pair_edge_pct=45" "pair_edge_pct=25" "pair_edge_pct=70" "pair_wps=1" "pair_wps=3" "march_min_th=48"; do
    tag=$(echo "$c $t" | tr ' =' '__')
    timeout -k 10 200 python3 -u bench.py $A --case $c --tune $t > $D/$tag.json 2> $D/$tag.err || exit 1
    python3 -c "
import json; d=json.load(open('$D/$tag.json')); r=d['roofline']
print('$c $t', r['avg_launch_us'], 'us/launch', round(r['avg_launch_us']/r['sweeps_per_launch'],2), 'us/sweep')"
  done
done
