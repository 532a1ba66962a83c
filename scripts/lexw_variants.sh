#!/usr/bin/env bash
# A/B of library build variants (CFD_AMD_LIB) x sweeps per launch, lex ordering, 4096^2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in ${LIBS:-libcfd_amd.so}; do
  for ns in ${NS_LIST:-2 3}; do
    CFD_AMD_LIB=$lib timeout -k 10 120 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --ordering lex --sweeps-per-launch $ns > gpurun_out/v_${lib}_$ns.json 2> gpurun_out/v_${lib}_$ns.err
    rc=$?; if [ $rc -ne 0 ]; then echo "$lib ns=$ns exit $rc"; tail -3 gpurun_out/v_${lib}_$ns.err; exit $rc; fi
    python3 -c "import json; d=json.load(open('gpurun_out/v_${lib}_$ns.json')); r=d['roofline']; print('$lib ns=$ns', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'])"
  done
done
