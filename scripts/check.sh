#!/usr/bin/env bash
# GPU suite + smoke + default bench line on one GPU; stops at the first failure.
# OUT (default gpurun_out/check) collects the logs; PYTEST_ARGS narrows the suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/check}
mkdir -p $F
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1200 python -u -m pytest -x -v --timeout 300 --timeout-method thread ${TESTS:-tests} -m gpu ${PYTEST_ARGS:-} > $F/pytest_gpu.log 2>&1
  rc=$?; echo "pytest exit $rc"; tail -n 4 $F/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1
  rc=$?; echo "smoke exit $rc"; tail -n 2 $F/smoke.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 300 python3 -u bench.py ${BENCH_ARGS:-} > $F/bench.json 2> $F/bench.err
  rc=$?; echo "bench exit $rc"; cat $F/bench.json; [ $rc -ne 0 ] && { tail -5 $F/bench.err; exit $rc; }
fi
exit 0
