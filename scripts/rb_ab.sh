#!/usr/bin/env bash
# A/B of library builds (CFD_AMD_LIB) on the red-black bench (4096^2 cavity).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in ${LIBS:-libcfd_amd.so}; do
  CFD_AMD_LIB=$lib timeout -k 10 120 python3 -u bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline ${EXTRA:-} > gpurun_out/rb_$lib.json 2> gpurun_out/rb_$lib.err
  rc=$?; if [ $rc -ne 0 ]; then echo "$lib exit $rc"; tail -3 gpurun_out/rb_$lib.err; exit $rc; fi
  python3 -c "import json; d=json.load(open('gpurun_out/rb_$lib.json')); r=d['roofline']; print('$lib', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'])"
done
