#!/usr/bin/env bash
# Round-5 GPU batch 9: the channel's red-black order on the resident launch -
# bit tests, the whole resident file (the kernel changed for every case), then
# the configs[2] red-black bench resident vs march.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b9; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_resident.py > $D/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "PASS|FAIL|Error|error" $D/pytest.log | tail -n 30; [ $rc -ne 0 ] && exit $rc
for r in 1 0; do
  timeout -k 10 300 python3 -u bench.py --case channel --nx 4096 --ny 512 --ordering rb --steps 2 --warmup 1 \
    --no-cpu-baseline --tune resident=$r > $D/bench_rb_res$r.json 2> $D/bench_rb_res$r.err || exit $?
  cat $D/bench_rb_res$r.json
done
