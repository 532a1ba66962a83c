#!/usr/bin/env bash
# Round-5 GPU batch 16: ghost-column fix-ups behind tile-uniform branches - resident
# tests, then the channel (both orders) and cavity 1024^2 benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b17; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_resident.py > $D/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -n 2 $D/pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $D/pytest.log | head; exit $rc; }
for c in "channel 4096 512 lex" "channel 4096 512 rb" "cavity 1024 1024 rb" "cavity 1024 1024 lex"; do
  set -- $c
  timeout -k 10 300 python3 -u bench.py --case $1 --nx $2 --ny $3 --ordering $4 --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0 > $D/bench_$1_$4.json 2>> $D/err.log || exit $?
  python3 -c "import json;d=json.load(open('$D/bench_$1_$4.json'));print('$c',d['value'],d['ms_per_step'],d['roofline'].get('us_per_sweep'))"
done
