#!/usr/bin/env bash
# Reference-order (lex) open cases at the BASELINE sizes: one timestep each
# (capped at 10000 sweeps) for several ramp band floors
# (CFD_TUNE_LEXW_RAMP_PCT) - bench.py lines into $D.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${OUT:-gpurun_out/lex_ramp}; mkdir -p $D
for w in "channel:4096:512:1000" "backwards_step:8192:512:400"; do
  IFS=: read -r c nx ny re <<< "$w"
  for pct in ${PCTS:-0 50 100}; do
    timeout -k 10 120 python3 bench.py --case $c --nx $nx --ny $ny --re $re --ordering lex --steps 1 --warmup 1 \
      --no-cpu-baseline --lex-steps 0 --tune lexw_ramp_pct=$pct > $D/${c}_ramp$pct.json 2> $D/${c}_ramp$pct.err || exit 1
    python3 -c "import json,sys;d=json.load(open('$D/${c}_ramp$pct.json'));print('$c', $pct, d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_us'])"
  done
done
