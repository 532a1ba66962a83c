#!/usr/bin/env bash
# FETCH_SIZE / WRITE_SIZE of the SOR kernel per knob config (one rocprofv3 pass each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmcs
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    SWEEP_ITERS=20 timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/pmcs/$i-$c -o run --output-format csv -- python3 scripts/sweep_poisson.py $cfg > gpurun_out/pmcs/$i-$c.out 2> gpurun_out/pmcs/$i-$c.err
    rc=$?; echo "cfg $cfg $c exit $rc"; if [ $rc -ne 0 ]; then tail -3 gpurun_out/pmcs/$i-$c.err; exit $rc; fi
  done
  i=$((i+1))
done
