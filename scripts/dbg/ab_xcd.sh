set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lex_digests.py > gpurun_out/ab3_tests.log 2>&1 || { tail -30 gpurun_out/ab3_tests.log; exit 1; }
tail -2 gpurun_out/ab3_tests.log
for v in 1 0 1 0; do
  timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --lex-steps 0 --tune lexw_xband=$v > gpurun_out/ab3_b$v.json 2> gpurun_out/ab3_b$v.err || { tail gpurun_out/ab3_b$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab3_b$v.json')); r=d['roofline']; print('xband=$v', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'])"
done
