#!/usr/bin/env bash
# Round-end measurements: the default bench under rocprofv3 kernel-trace stats,
# SQ counters of both SOR kernels, the small-grid timing. Results under
# gpurun_out/final (copied to profiles/ by hand).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=gpurun_out/final
mkdir -p $F
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $F/bench -o run --output-format csv -- python3 bench.py > $F/bench.json 2> $F/bench.err
rc=$?; echo "bench exit $rc"; [ $rc -ne 0 ] && { tail -5 $F/bench.err; exit $rc; }
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
for o in rb lex; do
  timeout -s KILL 150 rocprofv3 --pmc $C -d $F/sq_$o -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --max-iters 6000 --no-cpu-baseline --lex-steps 0 --ordering $o --sweeps-per-launch 3 > $F/sq_$o.out 2> $F/sq_$o.err
  rc=$?; echo "sq $o exit $rc"; [ $rc -ne 0 ] && { tail -5 $F/sq_$o.err; exit $rc; }
done
timeout -k 10 400 python3 -u scripts/small_grid_timing.py > $F/small_grid_timing.json
rc=$?; echo "small exit $rc"; exit $rc
