#!/usr/bin/env bash
# Parity tests of the default SOR kernel, then a knob sweep on the bench grid.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "${PYTEST_K:-poisson or run_matches or strips or backstep}" > gpurun_out/pytest_sweep.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -n 4 gpurun_out/pytest_sweep.log
if grep -qE "illegal memory access|MEMORY_APERTURE|HSA_STATUS_ERROR" gpurun_out/pytest_sweep.log; then echo "GPU fault -- stopping"; exit 3; fi
if [ "$rc" -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python3 -u scripts/sweep_poisson.py "$@" 2>&1 | tee gpurun_out/sweep.log
