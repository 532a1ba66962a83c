#!/usr/bin/env bash
# A/B of bench configurations on one GPU: each line of $CONFIGS (';'-separated
# argument sets) runs bench.py once; outputs gpurun_out/ab_<n>.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra CFG <<< "${CONFIGS:---steps 3 --warmup 1 --no-cpu-baseline}"
n=0
for a in "${CFG[@]}"; do
  timeout -k 10 240 python3 -u bench.py $a > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err
  rc=$?; echo "[$n] $a -> exit $rc"; cat gpurun_out/ab_$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'])"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_$n.err; exit $rc; fi
  n=$((n+1))
done
