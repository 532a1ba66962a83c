#!/usr/bin/env bash
# GPU check for the Rayleigh-Benard case + regression subset + benches (metric line and RB extra line).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rayleigh_benard.py ${EXTRA_TESTS:-} -m gpu > gpurun_out/pytest_rb.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -n 12 gpurun_out/pytest_rb.log
if grep -qE "illegal memory access|MEMORY_APERTURE|HSA_STATUS_ERROR" gpurun_out/pytest_rb.log; then echo "GPU fault -- stopping"; exit 3; fi
if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-seconds 12 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench.err; exit $rc; fi
timeout -k 10 300 python -u bench.py --case rayleigh_benard --nx 8192 --ny 2048 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_rb.json 2> gpurun_out/bench_rb.err
rc=$?; echo "bench rb exit $rc"; cat gpurun_out/bench_rb.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_rb.err; exit $rc; fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
rc=$?; echo "rocprof exit $rc"; find gpurun_out/prof -name "*stats*" | head
