set -o pipefail
D=gpurun_out/ns6b; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_resident.py > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for c in "cavity --nx 1024 --ny 1024" "channel --nx 4096 --ny 512"; do
  n=${c%% *}
  for o in lex rb; do
    timeout -k 10 200 python -u bench.py --case $c --ordering $o --steps 3 --warmup 1 --no-cpu-baseline --lex-steps 0 > $D/$n$o.json 2> $D/$n$o.err || { tail $D/$n$o.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/$n$o.json')); r=d['roofline']; print('$n $o', round(d['value']), d['ms_per_step'], r.get('us_per_sweep'), d.get('proof_fallbacks'))"
  done
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/full.log 2>&1 || { tail -30 $D/full.log; exit 1; }
tail -1 $D/full.log
