set -o pipefail
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lexw.py tests/test_gpu_lex_digests.py tests/test_gpu_lex_ranks.py > gpurun_out/ab2_tests.log 2>&1 || { tail -30 gpurun_out/ab2_tests.log; exit 1; }
tail -2 gpurun_out/ab2_tests.log
for v in 1 0 1 0; do
  timeout -k 10 200 python -u bench.py --case backwards_step --nx 8192 --ny 512 --re 400 --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0 --tune lexw_updown=$v > gpurun_out/ab2_b$v.json 2> gpurun_out/ab2_b$v.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab2_b$v.json')); r=d['roofline']; print('step updown=$v', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'])"
done
