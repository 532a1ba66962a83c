#!/usr/bin/env bash
# Round-5 GPU batch 25: ramp-launch wall tiles on the unmasked march when
# wholly active (product) vs always masked (variant library), same box:
# cavity 4096^2 and step 8192x512 in the reference order.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b25; mkdir -p $D
K="--ordering lex --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0"
S="--case backwards_step --nx 8192 --ny 512 --re 400 $K"
for v in main ref0 main ref0; do
  if [ $v = ref0 ]; then export CFD_AMD_LIB=$PWD/computational-fluid-dynamics_amd/libcfd_amd_ref0.so; else unset CFD_AMD_LIB; fi
  for c in K S; do
    timeout -k 10 300 python3 -u bench.py ${!c} > $D/${v}_$c.json 2>> $D/err.log || exit $?
    python3 -c "import json;d=json.load(open('$D/${v}_$c.json'));print('$v','$c',d['value'],d['ms_per_step'])"
  done
done
