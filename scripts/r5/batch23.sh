#!/usr/bin/env bash
# Round-5 GPU batch 23: the step's reference-order evidence after the ramp
# floor default (bench, rocprofv3 kernel stats, PMC traffic).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
CASES="stlex" bash scripts/profile_round.sh > gpurun_out/prof/round_b23.log 2>&1
rc=$?; echo "profile exit $rc"; grep -E "exit|hbm_bytes|traffic_over" gpurun_out/prof/round_b23.log | head; exit $rc
