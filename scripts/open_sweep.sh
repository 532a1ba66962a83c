#!/usr/bin/env bash
# Open-case SOR launch time vs tiling knobs (channel 4096x512, step 8192x512).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/open
for c in ${CASES:-channel backwards_step}; do
  if [ $c = channel ]; then A="--case channel --nx 4096 --ny 512"; else A="--case backwards_step --nx 8192 --ny 512 --re 400"; fi
  for v in ${VALS:-24}; do
    env ${KNOB:-CFD_MARCH_MIN_TH}=$v timeout -k 10 120 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lex-steps 0 $A > gpurun_out/open/${c}_$v.json 2> gpurun_out/open/${c}_$v.err
    rc=$?; if [ $rc -ne 0 ]; then echo "$c $v exit $rc"; tail -3 gpurun_out/open/${c}_$v.err; exit $rc; fi
    python3 -c "import json; d=json.load(open('gpurun_out/open/${c}_$v.json')); r=d['roofline']; print('$c ${KNOB:-CFD_MARCH_MIN_TH}=$v', d['ms_per_step'], r['avg_launch_us'], r['frac'])"
  done
done
