#!/usr/bin/env bash
# Proof-mode convergence test on one GPU: its parity tests (and the launch-plan
# tests around it), the bench with and without it, and rocprofv3 kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/proof
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  ${PROOF_TESTS:-tests/test_gpu_proof.py tests/test_gpu_pairs.py tests/test_gpu_fullsize.py tests/test_gpu_ranks.py} > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -n 15 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --lex-steps 0 ${BENCH_ARGS:-} > $O/bench_proof.json 2> $O/bench_proof.err
rc=$?; echo "bench exit $rc"; cat $O/bench_proof.json; [ $rc -ne 0 ] && { tail -5 $O/bench_proof.err; exit $rc; }
CFD_PROOF=0 timeout -k 10 300 python3 -u bench.py --lex-steps 0 --no-cpu-baseline > $O/bench_exact.json 2> $O/bench_exact.err
rc=$?; echo "bench exact exit $rc"; cat $O/bench_exact.json; [ $rc -ne 0 ] && { tail -5 $O/bench_exact.err; exit $rc; }
CFD_PROOF_NS=4 timeout -k 10 300 python3 -u bench.py --lex-steps 0 --no-cpu-baseline > $O/bench_proof4.json 2> $O/bench_proof4.err
rc=$?; echo "bench proof4 exit $rc"; cat $O/bench_proof4.json; [ $rc -ne 0 ] && { tail -5 $O/bench_proof4.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0 > $O/prof.json 2> $O/prof.err
rc=$?; echo "rocprof exit $rc"; [ $rc -ne 0 ] && { tail -5 $O/prof.err; exit $rc; }
find $O/prof -name "*kernel_stats.csv" | head -3
