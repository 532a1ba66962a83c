#!/usr/bin/env bash
# Round-5 GPU batch 22: the step's crossing-tile bands in 3 (product) vs 6
# parts (variant library), same box; step tests on the variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b22; mkdir -p $D
S="--case backwards_step --nx 8192 --ny 512 --re 400 --ordering lex --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0"
for v in main xs6 main xs6; do
  if [ $v = xs6 ]; then export CFD_AMD_LIB=$PWD/computational-fluid-dynamics_amd/libcfd_amd_xs6.so; else unset CFD_AMD_LIB; fi
  timeout -k 10 300 python3 -u bench.py $S > $D/$v.json 2>> $D/err.log || exit $?
  python3 -c "import json;d=json.load(open('$D/$v.json'));print('$v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'])"
done
export CFD_AMD_LIB=$PWD/computational-fluid-dynamics_amd/libcfd_amd_xs6.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_lexw.py tests/test_gpu_lex_digests.py -k "step or digest" > $D/pytest_xs6.log 2>&1
rc=$?; echo "pytest xs6 exit $rc"; tail -n 1 $D/pytest_xs6.log; exit $rc
