#!/usr/bin/env bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_lexw.py > gpurun_out/lexw.log 2>&1
rc=$?; tail -n 30 gpurun_out/lexw.log; exit $rc
