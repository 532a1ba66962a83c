#!/usr/bin/env bash
# Open-case SOR: proof-mode 4-sweep march launches (open.hip) vs exact pair
# launches and the LDS tiles; tests first (stops at the first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${OUT:-gpurun_out/open_ab}
mkdir -p $D
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_open_proof.py ${EXTRA_TESTS:-} > $D/pytest.log 2>&1
  rc=$?; echo "pytest exit $rc"; tail -n 5 $D/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
A="--no-cpu-baseline --lex-steps 0 --steps ${STEPS:-2} --warmup 1"
run() {  # tag, args
  timeout -k 10 300 python3 -u bench.py $A $2 > $D/$1.json 2> $D/$1.err
  rc=$?; echo "$1 exit $rc"; python3 -c "
import json,sys; d=json.load(open('$D/$1.json')); r=d['roofline']
print('  ', d['value'], 'MLUPS', d['ms_per_step'], 'ms/step', r['kernel'], r['avg_launch_us'], 'us/launch', r['sweeps_per_launch'], 'sweeps/launch', round(r['avg_launch_us']/r['sweeps_per_launch'],2), 'us/sweep', 'fallbacks', d['proof_fallbacks'])" || true
  return $rc
}
CH="--case channel --nx 4096 --ny 512"; ST="--case backwards_step --nx 8192 --ny 512 --re 400"
run ch_march_proof "$CH --tile-rounds 0" && run ch_march_pairs "$CH --tile-rounds 0 --proof-test off" &&
run ch_tile "$CH" && run st_march_proof "$ST" && run st_march_pairs "$ST --proof-test off"
