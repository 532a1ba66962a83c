set -o pipefail
# Binade-chunked sequential sum: crafted-term tests, the reference-order parity
# suites that run the open cases' sums, then the two open-case benches in the
# reference order under a kernel trace (the sum's three kernels per step).
D=gpurun_out/seqsum; mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_seqsum.py > $D/t_seqsum.log 2>&1 || { tail -40 $D/t_seqsum.log; exit 1; }
tail -3 $D/t_seqsum.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_lex_digests.py tests/test_gpu_lex_ranks.py tests/test_gpu_binaries.py tests/test_gpu_baseline_configs.py > $D/t_lex.log 2>&1 || { tail -40 $D/t_lex.log; exit 1; }
tail -3 $D/t_lex.log
for c in "channel --nx 4096 --ny 512 --re 1000" "backwards_step --nx 8192 --ny 512 --re 400"; do
  n=${c%% *}
  timeout -k 10 300 python -u bench.py --case $c --steps 3 --warmup 1 --no-cpu-baseline --lex-steps 0 > $D/b_$n.json 2> $D/b_$n.err || { tail $D/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/b_$n.json')); print('$n', d['value'], d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 -u bench.py --case channel --nx 4096 --ny 512 --re 1000 --steps 3 --warmup 1 --no-cpu-baseline --lex-steps 0 > $D/prof.log 2>&1 || { tail $D/prof.log; exit 1; }
find $D/prof -name "*kernel_stats.csv" -exec cp {} $D/channel_kernel_stats.csv \;
grep -i "seq_" $D/channel_kernel_stats.csv || true
