#!/usr/bin/env bash
# One GPU call: the tests touched since the last full suite, stencil times,
# then the round profiles of the changed paths (stops at the first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/evidence; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_ranks.py} -m gpu > $D/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -n 3 $D/pytest.log; [ $rc -ne 0 ] && exit $rc
bash scripts/stencil_time.sh || exit 1
[ -n "$NO_PROFILE" ] && exit 0
CASES="${CASES:-cav1k ch st chlex}" bash scripts/profile_round.sh > $D/profile_round.log 2>&1
rc=$?; echo "profile exit $rc"; grep -E "exit|hbm_bytes|traffic_over" $D/profile_round.log | head -40; exit $rc
