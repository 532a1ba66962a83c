#!/usr/bin/env bash
# Round-5 GPU batch 18: check_every on the resident path, then the channel's
# round evidence (bench + rocprofv3 stats) with the latest resident kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b18; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_resident.py -k "check_every or lex" > $D/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "PASS|FAIL" $D/pytest.log | tail -n 6; [ $rc -ne 0 ] && { grep -E "Error|assert" $D/pytest.log | head; exit $rc; }
mkdir -p gpurun_out/prof
CASES="ch chlex cav1k cav1klex" bash scripts/profile_round.sh > gpurun_out/prof/round_b18.log 2>&1
rc=$?; echo "profile exit $rc"; grep -E "exit" gpurun_out/prof/round_b18.log | head; exit $rc
