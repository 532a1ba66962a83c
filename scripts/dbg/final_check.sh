set -o pipefail
# round-end rehearsal: the GPU suite, smoke(), the round's profiles, the default bench line
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_full.log 2>&1 || { tail -30 gpurun_out/final_full.log; exit 1; }
tail -1 gpurun_out/final_full.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { cat gpurun_out/final_smoke.log; exit 1; }
cat gpurun_out/final_smoke.log
rm -rf gpurun_out/prof
bash scripts/profile_round.sh > gpurun_out/profile_round.log 2>&1 || { tail -20 gpurun_out/profile_round.log; exit 1; }
echo profiles ok
timeout -k 10 300 python -u bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { tail gpurun_out/final_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/final_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic'), d.get('red_black', {}).get('value'), d['cpu_baseline'])"
