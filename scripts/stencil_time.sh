#!/usr/bin/env bash
# Stencil-kernel times (predictor, source, corrector, final residual) at the
# headline size: rocprofv3 kernel stats of short capped cavity steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=${OUT:-gpurun_out/stencil}; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/stats -o run --output-format csv -- python3 bench.py --no-cpu-baseline --lex-steps 0 --steps 4 --warmup 1 --max-iters 40 > $D/out.txt 2>&1 || exit 1
f=$(find $D/stats -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
mb = {"tentative_kernel": 537.3, "cavity_source_kernel": 403.0, "correct_kernel": 671.6, "cavity_resmax_kernel": 268.7}
for r in csv.DictReader(open(sys.argv[1])):
    for k, b in mb.items():
        if k in r["Name"]:
            us = float(r["AverageNs"]) / 1e3
            print(f"{k}: {us:.1f} us, {b / us * 1e-3:.2f} TB/s algorithmic = {b / us / 8000 * 1e3 / 1e3:.3f} of 8 TB/s")
PY
