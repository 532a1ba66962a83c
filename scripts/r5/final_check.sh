#!/usr/bin/env bash
# Round-5 round-end rehearsal on one GPU: the whole -m gpu suite, smoke(), and
# the default bench line (what the driver runs), each under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5final3; mkdir -p $D
timeout -k 10 1000 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -n 3 $D/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $D/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1
rc=$?; tail -n 2 $D/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u bench.py > $D/bench.json 2> $D/bench.err
rc=$?; echo "bench exit $rc"; cat $D/bench.json; exit $rc
