set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
D=gpurun_out/tile_prof; mkdir -p $D
A="--no-cpu-baseline --lex-steps 0 --steps 1 --warmup 1 --case channel --nx 4096 --ny 512"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/s4 -o run --output-format csv -- python3 bench.py $A > $D/s4.out 2>&1 && 
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/s1 -o run --output-format csv -- python3 bench.py $A --sweeps-per-launch 1 > $D/s1.out 2>&1 &&
for f in $(find $D -name '*kernel_stats.csv'); do echo $f; head -4 $f | cut -c1-250; done
