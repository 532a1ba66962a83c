#!/usr/bin/env bash
# SQ counters (one pass, <= 8 SQ counters) for the SOR kernels of the rb and
# lex orderings at 4096^2 (60 sweeps per step, one step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmcsq
export TMPDIR=/tmp
C="${PMC_COUNTERS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU}"
for o in ${ORDERS:-rb lex}; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmcsq/$o -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --max-iters ${PMC_ITERS:-60} --no-cpu-baseline --ordering $o ${EXTRA:-} > gpurun_out/pmcsq/$o.out 2> gpurun_out/pmcsq/$o.err
  rc=$?; echo "pmc $o exit $rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmcsq/$o.err; exit $rc; fi
done
find gpurun_out/pmcsq -name "*counter_collection.csv"
