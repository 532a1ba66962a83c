#!/usr/bin/env bash
# HBM traffic of the SOR kernel from PMC counters, one counter group per pass
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --max-iters ${PMC_ITERS:-100} --no-cpu-baseline"
for c in ${PMC_SETS:-FETCH_SIZE WRITE_SIZE}; do
  timeout -s KILL 240 rocprofv3 --pmc $c -d gpurun_out/pmc/$c -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/$c.out 2> gpurun_out/pmc/$c.err
  rc=$?; echo "pmc $c exit $rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/$c.err; exit $rc; fi
done
