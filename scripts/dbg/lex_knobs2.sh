set -o pipefail
run() {
  timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0 "$@" > gpurun_out/kn.json 2> gpurun_out/kn.err || { tail -3 gpurun_out/kn.err; return 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/kn.json')); r=d['roofline']; print(' '.join(sys.argv[1:]), d['value'], d['ms_per_step'], r['avg_launch_us'])" "$@"
}
run --sweeps-per-launch 5 || exit 1
run --sweeps-per-launch 3
run
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/kn5 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --lex-steps 0 --sweeps-per-launch 5 > /dev/null 2>&1
find gpurun_out/kn5 -name '*kernel_stats.csv' -exec head -3 {} \;
