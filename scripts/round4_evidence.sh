#!/usr/bin/env bash
# Round 4 evidence (one GPU call): the default bench line (cavity 4096^2
# red-black headline, the reference order beside it, the CPU legs), then the
# per-workload profiles (bench line, rocprofv3 kernel stats, PMC traffic).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/r4; mkdir -p $D
timeout -k 10 300 python3 -u bench.py > $D/bench_default.json 2> $D/bench_default.err
rc=$?; echo "bench exit $rc"; cat $D/bench_default.json; [ $rc -ne 0 ] && exit $rc
CASES="${CASES:-cav4k cav4klex chlex stlex cav1k ch st}" bash scripts/profile_round.sh > $D/profile_round.log 2>&1
rc=$?; echo "profile exit $rc"; grep -E "exit|hbm_bytes|traffic_over" $D/profile_round.log | head -60; exit $rc
