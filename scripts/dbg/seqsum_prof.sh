set -o pipefail
# kernel trace of the two open cases' reference-order benches (the sequential
# sum's kernels per step) -> gpurun_out/seqsum/
D=gpurun_out/seqsum; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in "channel --nx 4096 --ny 512 --re 1000" "backwards_step --nx 8192 --ny 512 --re 400"; do
  n=${c%% *}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_$n -o run --output-format csv -- python3 -u bench.py --case $c --steps 3 --warmup 1 --no-cpu-baseline --lex-steps 0 > $D/prof_$n.log 2>&1 || { tail $D/prof_$n.log; exit 1; }
  find $D/prof_$n -name "*kernel_stats.csv" -exec cp {} $D/${n}_kernel_stats.csv \;
  grep -i "seq_\|Name" $D/${n}_kernel_stats.csv | cut -c1-200
done
