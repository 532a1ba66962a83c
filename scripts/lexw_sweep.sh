#!/usr/bin/env bash
# lexw tuning sweep: sweeps per launch x tiles per launch (CFD_LEXW_WAVES), 4096^2 cavity.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for ns in ${NS_LIST:-2 3}; do
  for w in ${W_LIST:-1024 2048 3072 4096}; do
    CFD_LEXW_WAVES=$w timeout -k 10 120 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --ordering lex --sweeps-per-launch $ns > gpurun_out/sw_${ns}_$w.json 2> gpurun_out/sw_${ns}_$w.err
    rc=$?; if [ $rc -ne 0 ]; then echo "ns=$ns w=$w exit $rc"; tail -3 gpurun_out/sw_${ns}_$w.err; exit $rc; fi
    python3 -c "import json; d=json.load(open('gpurun_out/sw_${ns}_$w.json')); r=d['roofline']; print('ns=$ns waves=$w', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'])"
  done
done
