#!/usr/bin/env bash
# Round-5 GPU batch 6: the resident solve in the reference's order - bit tests
# (vs lexw and vs the reference-loop oracle), timings vs the lexw march.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b6; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_resident.py > $D/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "PASS|FAIL|Error|error" $D/pytest.log | tail -n 12; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/r5/resdbg_lex.py > $D/resdbg_lex.txt 2>&1; rc=$?; cat $D/resdbg_lex.txt; exit $rc
