#!/usr/bin/env bash
# Round-5 GPU batch 10: resident tests (the channel's red-black order added),
# the step's reference-order tests (split crossing-tile bands) and digests,
# then benches: channel red-black resident vs march, step reference order.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b10; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_resident.py -k "channel_rb" > $D/pytest_res.log 2>&1
rc=$?; echo "pytest resident exit $rc"; grep -E "PASS|FAIL|Error|error" $D/pytest_res.log | tail -n 30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_lexw.py tests/test_gpu_lex_digests.py -k "step or digest" > $D/pytest_step.log 2>&1
rc=$?; echo "pytest step exit $rc"; grep -E "PASS|FAIL|Error|error" $D/pytest_step.log | tail -n 20; [ $rc -ne 0 ] && exit $rc
for r in 1 0; do
  timeout -k 10 300 python3 -u bench.py --case channel --nx 4096 --ny 512 --ordering rb --steps 2 --warmup 1 \
    --no-cpu-baseline --tune resident=$r > $D/bench_rb_res$r.json 2> $D/bench_rb_res$r.err || exit $?
  cat $D/bench_rb_res$r.json
done
timeout -k 10 300 python3 -u bench.py --case backwards_step --nx 8192 --ny 512 --re 400 --ordering lex --steps 2 --warmup 1 --no-cpu-baseline > $D/bench_step_lex.json 2> $D/bench_step_lex.err || exit $?
cat $D/bench_step_lex.json
