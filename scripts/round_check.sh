#!/usr/bin/env bash
# Round evidence on one GPU (stops at the first failure): the whole GPU test
# suite, smoke(), the default bench line, rocprofv3 kernel stats of the bench
# command, and the HBM traffic (PMC) of the headline SOR launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=gpurun_out/final
mkdir -p $F
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $F/pytest_gpu.log 2>&1
  rc=$?; echo "pytest exit $rc"; tail -n 4 $F/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1
  rc=$?; echo "smoke exit $rc"; tail -n 2 $F/smoke.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python3 -u bench.py > $F/bench.json 2> $F/bench.err
rc=$?; echo "bench exit $rc"; cat $F/bench.json; [ $rc -ne 0 ] && { tail -5 $F/bench.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $F/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0 > $F/prof_bench.json 2> $F/prof_bench.err
rc=$?; echo "rocprof exit $rc"; [ $rc -ne 0 ] && { tail -5 $F/prof_bench.err; exit $rc; }
head -4 $F/prof/run_kernel_stats.csv
PMC_WARMUP=1 PMC_ITERS=400 ORDER=rb bash scripts/pmc_traffic.sh
