#!/usr/bin/env bash
# Round evidence on one GPU: bench line, rocprofv3 kernel-trace stats of the
# same command, and the two PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs)
# for the SOR kernel's HBM traffic. Post-process with scripts/pmc_summary.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench.err; exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof/bench_prof.json 2> gpurun_out/prof/bench_prof.err
rc=$?; echo "rocprof exit $rc"; cat gpurun_out/prof/bench_prof.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof/bench_prof.err; exit $rc; fi
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/pmc/$c -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --max-iters 100 --no-cpu-baseline > gpurun_out/pmc/$c.out 2> gpurun_out/pmc/$c.err
  rc=$?; echo "pmc $c exit $rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/$c.err; exit $rc; fi
done
find gpurun_out/prof gpurun_out/pmc -name "*.csv" | head -20
