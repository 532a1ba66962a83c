#!/usr/bin/env bash
# Round-5 GPU batch 8: where the backwards step's reference-order solve spends
# its time - per-launch wave stamps of lexw (diagnostic build), the bench line
# and a rocprofv3 kernel summary of the same workload.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b8; mkdir -p $D
CFD_AMD_LIB=$PWD/computational-fluid-dynamics_amd/libcfd_amd_lstamps.so timeout -k 10 240 python3 -u scripts/dbg/lexw_stamps.py backwards_step 8192 512 > $D/step_stamps.json 2> $D/step_stamps.err || exit $?
timeout -k 10 300 python3 -u bench.py --case backwards_step --nx 8192 --ny 512 --re 400 --ordering lex --steps 2 --warmup 1 --no-cpu-baseline > $D/bench_step_lex.json 2> $D/bench_step_lex.err || exit $?
cat $D/bench_step_lex.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o step -- python3 bench.py --case backwards_step --nx 8192 --ny 512 --re 400 --ordering lex --steps 2 --warmup 1 --no-cpu-baseline > $D/prof.log 2>&1 || exit $?
find $D/prof -name "*kernel_stats.csv" | head -3
