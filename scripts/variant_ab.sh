#!/usr/bin/env bash
# Bench lines of in-tree build variants (CFD_AMD_LIB) against the default
# library: VARIANTS="lib1 lib2 ..." (files in computational-fluid-dynamics_amd/),
# WORKLOADS="name:args;name:args" (stops at the first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${OUT:-gpurun_out/variant_ab}; mkdir -p $D
A="--no-cpu-baseline --lex-steps 0 --steps ${STEPS:-3} --warmup 1"
IFS=';' read -ra WL <<< "$WORKLOADS"
for w in "${WL[@]}"; do
  name=${w%%:*}; args=${w#*:}
  for lib in libcfd_amd.so $VARIANTS; do
    tag=${name}_${lib%.so}
    CFD_AMD_LIB=$lib timeout -k 10 300 python3 -u bench.py $A $args > $D/$tag.json 2> $D/$tag.err || { tail -3 $D/$tag.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$D/$tag.json')); r=d['roofline']
print('$tag', d['value'], 'MLUPS', r['avg_launch_us'], 'us/launch', round(r['avg_launch_us']/r['sweeps_per_launch'],2), 'us/sweep', 'frac', r['frac'])"
  done
done
