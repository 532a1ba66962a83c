#!/usr/bin/env bash
# HBM traffic of the SOR launches at 4096^2 (FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 passes; MI355X_MICROARCH.md HBM [CDNA4]): the red-black
# kernel of the headline (ORDER=rb) or the lexicographic kernel (ORDER=lex,
# steady launches only). scripts/pmc_traffic.py turns the CSVs into JSON.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${ORDER:-rb}
D=gpurun_out/pmctraffic/$O
mkdir -p $D
export TMPDIR=/tmp
A="--steps 1 --warmup ${PMC_WARMUP:-0} --max-iters ${PMC_ITERS:-100} --no-cpu-baseline --lex-steps 0 --ordering $O --sweeps-per-launch 3"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c -d $D/$c -o run --output-format csv -- python3 bench.py $A > $D/$c.out 2> $D/$c.err
  rc=$?; echo "pmc $O $c exit $rc"; if [ $rc -ne 0 ]; then tail -5 $D/$c.err; exit $rc; fi
done
