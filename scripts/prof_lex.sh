#!/usr/bin/env bash
# rocprofv3 kernel-trace stats of one lex-ordered bench step (4096^2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/${OUT:-proflex}
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${OUT:-proflex} -o run --output-format csv -- python3 bench.py --steps ${STEPS:-1} --warmup 1 --no-cpu-baseline --ordering ${ORDER:-lex} ${EXTRA:-} > gpurun_out/${OUT:-proflex}/bench.json 2> gpurun_out/${OUT:-proflex}/bench.err
rc=$?; echo "rocprof exit $rc"; cat gpurun_out/${OUT:-proflex}/bench.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/${OUT:-proflex}/bench.err; exit $rc; fi
f=$(find gpurun_out/${OUT:-proflex} -name "*kernel_stats.csv" | head -1); echo $f; head -12 $f
