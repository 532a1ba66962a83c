#!/usr/bin/env bash
# SQ counters of the lexw kernels at 1024^2 (2000 sweeps: ramps and a steady
# phase), normal run (n) and with every launch on the ramp kernel (r).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmcramp
export TMPDIR=/tmp
C="${PMC_COUNTERS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU}"
A="--nx 1024 --ny 1024 --steps 1 --warmup 0 --max-iters 2000 --no-cpu-baseline --ordering lex --sweeps-per-launch ${NS:-2}"
timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmcramp/n -o run --output-format csv -- python3 bench.py $A > gpurun_out/pmcramp/n.out 2> gpurun_out/pmcramp/n.err
rc=$?; echo "pmc n exit $rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmcramp/n.err; exit $rc; fi
export CFD_LEXW_RAMP_KERNEL=1
timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmcramp/r -o run --output-format csv -- python3 bench.py $A > gpurun_out/pmcramp/r.out 2> gpurun_out/pmcramp/r.err
rc=$?; echo "pmc r exit $rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmcramp/r.err; exit $rc; fi
find gpurun_out/pmcramp -name "*counter_collection.csv"
