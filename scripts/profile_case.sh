#!/usr/bin/env bash
# Evidence for one workload on one GPU (stops at the first failure): the bench
# line, rocprofv3 kernel stats of the same command, and the HBM traffic of its
# SOR launch (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md
# HBM [CDNA4]; scripts/pmc_traffic.py applies the gfx950 corrections).
#   CASE NX NY RE ORDER (rb|lex)  KSUB = the SOR kernel's name substring
#   SPL = its sweeps per launch   PMC_ITERS = the capped solve the PMC passes time
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-${CASE}_${ORDER}_${NX}x${NY}}
D=gpurun_out/prof/$TAG
mkdir -p $D
export TMPDIR=/tmp
A="--case $CASE --nx $NX --ny $NY --re ${RE:-1000} --ordering $ORDER --no-cpu-baseline --lex-steps 0 ${EXTRA}"
W="--warmup ${PMC_WARMUP:-1}"  # (the first step: source in the lid corners only, not the steady state)
timeout -k 10 300 python3 -u bench.py $A --steps ${STEPS:-2} --warmup 1 > $D/bench.json 2> $D/bench.err
rc=$?; echo "bench exit $rc"; cat $D/bench.json; [ $rc -ne 0 ] && { tail -5 $D/bench.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/stats -o run --output-format csv -- python3 bench.py $A --steps 1 --warmup 1 > $D/stats.out 2> $D/stats.err
rc=$?; echo "rocprof exit $rc"; [ $rc -ne 0 ] && { tail -5 $D/stats.err; exit $rc; }
find $D/stats -name '*kernel_stats.csv' -exec head -4 {} \;
[ -n "$NO_PMC" ] && exit 0  # (the resident whole-solve launch: no per-sweep HBM stream to count)
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c -d $D/$c -o run --output-format csv -- python3 bench.py $A --steps 1 $W --max-iters ${PMC_ITERS:-400} > $D/$c.out 2> $D/$c.err
  rc=$?; echo "pmc $c exit $rc"; [ $rc -ne 0 ] && { tail -5 $D/$c.err; exit $rc; }
done
python3 scripts/pmc_traffic.py $D "$KSUB" $D/pmc.json $NX $SPL $NY > /dev/null && echo "pmc ok" && grep -E "hbm_bytes_per_launch|traffic_over" $D/pmc.json
