#!/usr/bin/env bash
# The reference order's sequential source sum chained over ranks (channel
# 4096x512, one step on 1 GPU and on 4 loopback ranks sharing it): rocprofv3
# kernel stats of the sum's kernels (seq_approx / seq_units / seq_chunk /
# seq_walk_kernel: each rank evaluates its own terms' chunks, the walks chain
# rank to rank) -> gpurun_out/seqsum_ranks/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/seqsum_ranks; mkdir -p $D
A="--case channel --nx 4096 --ny 512 --ordering lex --steps 1 --warmup 1 --no-cpu-baseline --lex-steps 0 --max-iters 200"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/one -o run --output-format csv -- python3 bench.py $A > $D/one.json 2> $D/one.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/four -o run --output-format csv -- python3 bench.py $A --loopback-ranks 4 > $D/four.json 2> $D/four.err || exit 1
for r in one four; do echo $r; find $D/$r -name '*kernel_stats.csv' -exec grep -h "seq_" {} \; ; done
