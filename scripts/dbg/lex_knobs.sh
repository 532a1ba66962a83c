# A/B of the reference-order launch plan at 4096^2 after the up/down split (bench value, steady launch)
set -o pipefail
run() {
  timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0 "$@" > gpurun_out/kn.json 2> gpurun_out/kn.err || { tail -3 gpurun_out/kn.err; return 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/kn.json')); r=d['roofline']; print(' '.join(sys.argv[1:]), d['value'], d['ms_per_step'], r['avg_launch_us'])" "$@"
}
run || exit 1
run --lex-sweeps 5
run --tune lexw_waves=1536
run --tune lexw_waves=2560
run --tune lexw_waves=3072
run --tune lexw_edge_pct=75
run --tune lexw_ramp_pct=50
run --tune march_min_th=24
run
