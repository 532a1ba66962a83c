#!/usr/bin/env bash
# tentative_kernel time vs band height (CFD_TENT_TH), 4096^2 cavity, 30-sweep steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tent
export TMPDIR=/tmp
for th in ${VALS:-16 32 64 128}; do
  CFD_TENT_TH=$th timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/tent/$th -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --lex-steps 0 --max-iters 30 > gpurun_out/tent/$th.json 2> gpurun_out/tent/$th.err
  rc=$?; if [ $rc -ne 0 ]; then echo "th=$th exit $rc"; tail -3 gpurun_out/tent/$th.err; exit $rc; fi
  echo "th=$th $(grep tentative gpurun_out/tent/$th/run_kernel_stats.csv | cut -d, -f2-4)"
done
