#!/usr/bin/env bash
# A/B of library builds (scripts/build_variant.sh NAME FLAGS) on the bench:
# LIBS="default p55 ..." x NSS="3 4" (proof-mode sweeps per launch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for lib in ${LIBS:-default}; do
  for ns in ${NSS:-3 4}; do
    L=libcfd_amd_$lib.so; [ "$lib" = default ] && L=libcfd_amd.so
    CFD_AMD_LIB=$L CFD_PROOF_NS=$ns timeout -k 10 200 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0 ${BENCH_ARGS:-} > gpurun_out/ab/${lib}_$ns.json 2> gpurun_out/ab/${lib}_$ns.err
    rc=$?
    python3 -c "import json; d=json.load(open('gpurun_out/ab/${lib}_$ns.json')); r=d['roofline']; print('$lib', $ns, d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'])" || { tail -3 gpurun_out/ab/${lib}_$ns.err; }
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
