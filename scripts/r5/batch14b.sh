#!/usr/bin/env bash
# Round-5 GPU batch 14: phase stamps of the resident solve (diagnostic build)
# at the BASELINE sizes it serves: cavity 1024^2 rb / lex, channel 4096x512 rb / lex.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b14b; mkdir -p $D
export CFD_AMD_LIB=$PWD/computational-fluid-dynamics_amd/libcfd_amd_rstamps.so
for c in "4096 512 10000 channel lex" "4096 512 10000 channel rb" "1024 1024 10000 cavity lex"; do
  set -- $c
  timeout -k 10 240 python3 -u scripts/dbg/res_stamps.py $c > $D/stamps_$4_$5_$1x$2.json 2>> $D/err.log || exit $?
  python3 -c "import json;d=json.load(open('$D/stamps_$4_$5_$1x$2.json'));print('$c', d['us_per_sweep'], {k:v for k,v in d.items() if k.endswith('_mean')})"
done
