#!/usr/bin/env bash
# Round-5 GPU batch 21: waves in flight for the reference-order march
# (lexw_waves) at the step's 8192x512 and the cavity's 4096^2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b21; mkdir -p $D
S="--case backwards_step --nx 8192 --ny 512 --re 400 --ordering lex --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0"
K="--ordering lex --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0"
for w in 2048 1536 2560 3072 2048; do
  for c in S K; do
    timeout -k 10 300 python3 -u bench.py ${!c} --tune lexw_waves=$w > $D/$c$w.json 2>> $D/err.log || exit $?
    python3 -c "import json;d=json.load(open('$D/$c$w.json'));print('$c',$w,d['value'],d['ms_per_step'])"
  done
done
