#!/usr/bin/env bash
# Bench the open cases (extra measurements, not the metric line): library variants A/B.
# LIBS="libcfd_amd.so libcfd_amd_x.so" bash scripts/case_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in ${LIBS:-libcfd_amd.so}; do
  for cfg in "channel 4096 512" "backwards_step 8192 512"; do
    set -- $cfg
    CFD_AMD_LIB=$L timeout -k 10 300 python -u bench.py --case $1 --nx $2 --ny $3 --steps 1 --warmup 1 --max-iters ${ITERS:-2000} --no-cpu-baseline > gpurun_out/case_$1.json 2> gpurun_out/case_$1.err
    rc=$?; if [ $rc -ne 0 ]; then tail -5 gpurun_out/case_$1.err; exit $rc; fi
    python3 -c "import json;d=json.load(open('gpurun_out/case_$1.json'));r=d['roofline'];print('$L $1', d['value'], 'MLUPS', r['avg_launch_us'], 'us/launch', r['sweeps_per_launch'], 'sweeps/launch', d['sor_iterations_per_step'])"
  done
done
