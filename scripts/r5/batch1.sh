#!/usr/bin/env bash
# Round-5 GPU batch 1: add-chain latency floor, new tests (RCCL send/recv to
# self, smlex MAXC 4/5, steady reference-order digests), the sequential-sum
# rewrite (timing + the open cases' reference-order bit tests), default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b1; mkdir -p $D
timeout -k 10 60 tools/add_chain > $D/add_chain.json 2>&1
rc=$?; echo "add_chain exit $rc"; cat $D/add_chain.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rccl.py \
  tests/test_gpu_smlex.py tests/test_gpu_lex_digests.py -k "not fixture_present" > $D/pytest1.log 2>&1
rc=$?; echo "pytest1 exit $rc"; tail -n 3 $D/pytest1.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/seqsum_timing.py > $D/seqsum.json 2> $D/seqsum.err
rc=$?; echo "seqsum exit $rc"; cat $D/seqsum.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_lexw.py \
  tests/test_gpu_lex.py -k "channel or step" > $D/pytest2.log 2>&1
rc=$?; echo "pytest2 exit $rc"; tail -n 3 $D/pytest2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err
rc=$?; echo "bench exit $rc"; cat $D/bench.json; exit $rc
