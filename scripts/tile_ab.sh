#!/usr/bin/env bash
# LDS-tile SOR launches vs the wave march: tile tests, then bench lines of the
# open-case and 1024^2 configs both ways (stops at the first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${OUT:-gpurun_out/tile_ab}
mkdir -p $D
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_tile.py ${EXTRA_TESTS:-} > $D/pytest.log 2>&1
  rc=$?; echo "pytest exit $rc"; tail -n 5 $D/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
A="--no-cpu-baseline --lex-steps 0 --steps ${STEPS:-2} --warmup 1"
run() {  # tag, args [, library file: an in-tree build variant]
  CFD_AMD_LIB=${3:-libcfd_amd.so} timeout -k 10 300 python3 -u bench.py $A $2 > $D/$1.json 2> $D/$1.err
  rc=$?; echo "$1 exit $rc"; python3 -c "
import json,sys; d=json.load(open('$D/$1.json')); r=d['roofline']
print('  ', d['value'], 'MLUPS', d['ms_per_step'], 'ms/step', r['kernel'], r['avg_launch_us'], 'us/launch', r['sweeps_per_launch'], 'sweeps/launch', round(r['avg_launch_us']/r['sweeps_per_launch'],2), 'us/sweep')" || true
  return $rc
}
CH="--case channel --nx 4096 --ny 512"; CV="--case cavity --nx 1024 --ny 1024"
if [ -n "$SLOPE" ]; then  # launch time vs sweeps per launch: per-sweep cost and fixed cost
  for n in 1 2 3; do run ch_spl$n "$CH --sweeps-per-launch $n" && run cv_spl$n "$CV --sweeps-per-launch $n" || exit 1; done
  run ch_spl4 "$CH" && run cv_spl4 "$CV"; exit $?
fi
run ch_tile "$CH" && run ch_tile_b1 "$CH" libcfd_amd_b1.so && run ch_tile_exact "$CH --proof-test off" &&
run ch_march "$CH --tile-rounds 0" &&
run cav1k_tile "$CV" && run cav1k_tile_b1 "$CV" libcfd_amd_b1.so && run cav1k_tile_exact "$CV --proof-test off" &&
run cav1k_march "$CV --tile-rounds 0"
