#!/usr/bin/env bash
# Quick GPU iteration: selected GPU tests, then the bench in the given modes.
# TESTS="tests/test_gpu_pairs.py" BENCH_MODES="1 2" bash scripts/quick.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS > gpurun_out/pytest_quick.log 2>&1
  rc=$?; echo "pytest exit $rc"; tail -n 25 gpurun_out/pytest_quick.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
for m in ${BENCH_MODES:-}; do
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --sweeps-per-launch $m ${BENCH_EXTRA:-} > gpurun_out/bench_m$m.json 2> gpurun_out/bench_m$m.err
  rc=$?; echo "bench mode $m exit $rc"; cat gpurun_out/bench_m$m.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_m$m.err; exit $rc; fi
done
