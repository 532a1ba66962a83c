#!/usr/bin/env bash
# A/B of SOR kernel launch flags (diagnostic): bench once per CFD_MARCH_FLAGS value.
# FLAGS="3 19 35" SPL=2 bash scripts/flags_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for f in ${FLAGS:-3}; do
  CFD_MARCH_FLAGS=$f timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --max-iters ${ITERS:-2000} --no-cpu-baseline --sweeps-per-launch ${SPL:-2} ${BENCH_EXTRA:-} > gpurun_out/ab_$f.json 2> gpurun_out/ab_$f.err
  rc=$?; echo "flags $f exit $rc"; python3 -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));r=d['roofline'];print('flags $f', d['value'], 'MLUPS', r['avg_launch_us'], 'us/launch', r['sweeps_per_launch'], 'sweeps/launch')"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_$f.err; exit $rc; fi
done
