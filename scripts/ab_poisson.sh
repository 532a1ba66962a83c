#!/usr/bin/env bash
# A/B of the two SOR kernel variants on the bench workload + the Poisson parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "${PYTEST_K:-poisson or run_matches or strips or backstep}" > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -n 5 gpurun_out/pytest_ab.log
if grep -qE "illegal memory access|MEMORY_APERTURE|HSA_STATUS_ERROR" gpurun_out/pytest_ab.log; then echo "GPU fault -- stopping"; exit 3; fi
if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit $rc; fi
for v in ${VARIANTS:-march tile}; do
  CFD_POISSON_KERNEL=$v timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_EXTRA:-} > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err
  rc=$?; echo "bench $v exit $rc"; python3 -c "import json;d=json.load(open('gpurun_out/bench_$v.json'));print('$v', d['value'], d['roofline'])" || tail -3 gpurun_out/bench_$v.err
  if [ "$rc" -ne 0 ]; then exit $rc; fi
done
