#!/usr/bin/env bash
# Round-5 GPU batch 5: full GPU suite with the resident solve as the red-black
# cavity default, then the 1024^2 red-black bench line (resident vs tiles).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b5; mkdir -p $D
timeout -k 10 840 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > $D/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -n 5 $D/pytest.log; [ $rc -ne 0 ] && exit $rc
A="--no-cpu-baseline --lex-steps 0 --steps 3 --warmup 1 --nx 1024 --ny 1024"
for w in "res:--tune resident=1" "tile:--tune resident=0"; do
  name=${w%%:*}; args=${w#*:}
  timeout -k 10 300 python3 -u bench.py $A $args > $D/bench_$name.json 2> $D/bench_$name.err
  rc=$?; echo "bench $name exit $rc"; [ $rc -ne 0 ] && { tail -3 $D/bench_$name.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('$D/bench_$name.json'))
print('$name', d['value'], 'MLUPS', d['ms_per_step'], 'ms/step', d['roofline'].get('kernel'))"
done
