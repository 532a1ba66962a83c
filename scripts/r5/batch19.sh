#!/usr/bin/env bash
# Round-5 GPU batch 19: the step's reference order - ramp band floor and
# boundary band length knobs (A/B on one box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b19b; mkdir -p $D
A="--case backwards_step --nx 8192 --ny 512 --re 400 --ordering lex --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0"
for t in "lexw_ramp_pct=100" "lexw_ramp_pct=150" "lexw_ramp_pct=200" "lexw_ramp_pct=300" "lexw_ramp_pct=100"; do
  timeout -k 10 300 python3 -u bench.py $A --tune $t > $D/step_$t.json 2>> $D/err.log || exit $?
  python3 -c "import json;d=json.load(open('$D/step_$t.json'));print('$t',d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'])"
done
