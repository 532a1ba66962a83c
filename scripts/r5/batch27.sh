#!/usr/bin/env bash
# Round-5 GPU batch 27: the cavity 4096^2 reference order's ramp band floor
# after the ramp edge march change (A/B on one box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b27; mkdir -p $D
K="--ordering lex --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0"
for rp in 0 100 50 0 100; do
  timeout -k 10 300 python3 -u bench.py $K --tune lexw_ramp_pct=$rp > $D/rp$rp.json 2>> $D/err.log || exit $?
  python3 -c "import json;d=json.load(open('$D/rp$rp.json'));print('ramp_pct',$rp,d['value'],d['ms_per_step'])"
done
