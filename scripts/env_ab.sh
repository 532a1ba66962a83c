#!/usr/bin/env bash
# A/B of solver tuning switches on the bench: ENVS="A=1,B=2;A=3" (';' between
# runs, ',' between variables of one run); BENCH_ARGS extra bench arguments.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/envab
IFS=';' read -ra RUNS <<< "${ENVS:-}"
n=0
for e in "${RUNS[@]}"; do
  env $(echo "$e" | tr ',' ' ') timeout -k 10 200 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0 ${BENCH_ARGS:-} > gpurun_out/envab/$n.json 2> gpurun_out/envab/$n.err
  rc=$?
  python3 -c "import json; d=json.load(open('gpurun_out/envab/$n.json')); r=d['roofline']; print('[$e]', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'])" || tail -3 gpurun_out/envab/$n.err
  [ $rc -ne 0 ] && exit $rc
  n=$((n+1))
done
exit 0
