#!/usr/bin/env bash
# Round-5 GPU batch 2: the step's left-tile class in the reference-order march
# (bit tests, digests at full size, A/B vs the masked march), the unrolled
# sequential sum (timing + open-case reference-order tests), open-case lex bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b2; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_lex_digests.py \
  tests/test_gpu_lexw.py tests/test_gpu_lex.py > $D/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -n 3 $D/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/seqsum_timing.py > $D/seqsum.json 2> $D/seqsum.err
rc=$?; echo "seqsum exit $rc"; cat $D/seqsum.json; [ $rc -ne 0 ] && exit $rc
A="--no-cpu-baseline --lex-steps 0 --steps 2 --warmup 1 --ordering lex"
for w in "step:--case backwards_step --nx 8192 --ny 512 --re 400" "step_masked:--case backwards_step --nx 8192 --ny 512 --re 400 --tune lexw_left=0" "channel:--case channel --nx 4096 --ny 512"; do
  name=${w%%:*}; args=${w#*:}
  timeout -k 10 300 python3 -u bench.py $A $args > $D/bench_$name.json 2> $D/bench_$name.err
  rc=$?; echo "bench $name exit $rc"; [ $rc -ne 0 ] && { tail -3 $D/bench_$name.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('$D/bench_$name.json')); r=d['roofline']
print('$name', d['value'], 'MLUPS', d['ms_per_step'], 'ms/step', r['avg_launch_us'], 'us steady launch', 'frac', r['frac'])"
done
