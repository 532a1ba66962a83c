#!/usr/bin/env bash
# Round-5 GPU batch 15: the channel's red-black resident sweeps unrolled per
# full group (lean variant for interior waves) - tests, then A/B of the proof
# from one row per wave (product) vs every row (variant library).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b15; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_resident.py -k "channel_rb" > $D/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "passed|failed" $D/pytest.log | tail -n 2; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $D/pytest.log | head; exit $rc; }
A="--case channel --nx 4096 --ny 512 --ordering rb --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0"
for v in main all main all; do
  if [ $v = all ]; then export CFD_AMD_LIB=$PWD/computational-fluid-dynamics_amd/libcfd_amd_rproofall.so; else unset CFD_AMD_LIB; fi
  timeout -k 10 300 python3 -u bench.py $A > $D/bench_$v.json 2>> $D/err.log || exit $?
  python3 -c "import json;d=json.load(open('$D/bench_$v.json'));print('$v',d['value'],d['ms_per_step'],d['roofline']['us_per_sweep'],d['proof_fallbacks'])"
done
