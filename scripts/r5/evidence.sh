#!/usr/bin/env bash
# Round-5 evidence: scripts/profile_round.sh over the BASELINE configs on their
# default paths (bench line, rocprofv3 kernel stats, PMC HBM traffic where the
# path streams HBM per launch). CFD_COMMIT names the profiled tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
CASES="${CASES:-cav4k cav4klex stlex st cav1k cav1klex ch chlex}" bash scripts/profile_round.sh > gpurun_out/prof/round.log 2>&1
rc=$?; echo "profile exit $rc"; grep -E "exit|hbm_bytes|traffic_over" gpurun_out/prof/round.log | head -60; exit $rc
