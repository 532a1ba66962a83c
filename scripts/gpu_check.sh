#!/usr/bin/env bash
# GPU-box check: parity tests, smoke, short bench. Stops at the first step that
# dies abnormally (fault / abort / timeout), per the pool's rules.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok_or_stop() { # $1 = exit code, $2 = step name; pytest's 1 (= failures) is not abnormal
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "ABNORMAL exit $1 in $2 -- stopping"; exit "$1"; fi
}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -n 15 gpurun_out/pytest_gpu.log; ok_or_stop $rc pytest
if grep -qE "illegal memory access|MEMORY_APERTURE|HSA_STATUS_ERROR" gpurun_out/pytest_gpu.log; then echo "GPU fault in pytest -- stopping"; exit 3; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -n 3 gpurun_out/smoke.log; ok_or_stop $rc smoke
if [ "$rc" -ne 0 ]; then echo "smoke failed -- stopping"; exit 4; fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:---steps 2 --warmup 1 --cpu-seconds 5} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench.json; tail -n 5 gpurun_out/bench.err
if [ "$rc" -ne 0 ]; then exit "$rc"; fi
if [ -n "${PROFILE:-}" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
  rc=$?; echo "rocprof exit $rc"; find gpurun_out/prof -name "*stats*" | head; ok_or_stop $rc rocprof
fi
