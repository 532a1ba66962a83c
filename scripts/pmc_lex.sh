#!/usr/bin/env bash
# SQ counters of the lexw kernels at 4096^2 (one step capped at PMC_ITERS
# sweeps: ramps plus a steady phase). One pass per counter set.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmclex
export TMPDIR=/tmp
C="${PMC_COUNTERS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU}"
A="--steps 1 --warmup 0 --max-iters ${PMC_ITERS:-6000} --no-cpu-baseline --ordering ${ORDER:-lex} --sweeps-per-launch ${NS:-3}"
timeout -s KILL 150 rocprofv3 --pmc $C -d gpurun_out/pmclex/${TAG:-a} -o run --output-format csv -- python3 bench.py $A > gpurun_out/pmclex/${TAG:-a}.out 2> gpurun_out/pmclex/${TAG:-a}.err
rc=$?; echo "pmc exit $rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmclex/${TAG:-a}.err; fi; exit $rc
