#!/usr/bin/env bash
# Per-kernel times of the non-SOR stencils (rocprofv3 kernel stats) for
# settings ENVS="A=1;A=2" (';' between runs) and libraries LIBS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/stencil
IFS=';' read -ra RUNS <<< "${ENVS:-X=0}"
n=0
for lib in ${LIBS:-default}; do
  L=libcfd_amd_$lib.so; [ "$lib" = default ] && L=libcfd_amd.so
  for e in "${RUNS[@]}"; do
    D=gpurun_out/stencil/$n
    env $(echo "$e" | tr "," " ") CFD_AMD_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --max-iters 6 --no-cpu-baseline --lex-steps 0 > $D.out 2> $D.err
    rc=$?
    [ $rc -ne 0 ] && { echo "run $n ($lib $e) exit $rc"; tail -3 $D.err; exit $rc; }
    echo "[$lib $e]"; grep -E "tentative|source_kernel|resmax|correct_kernel|centers_stats|subtract_mean|bc_cavity" $D/run_kernel_stats.csv | awk -F',' '{gsub(/"/,"",$1); split($1,a,"("); printf "  %-40s %s\n", a[1], $4}'
    n=$((n+1))
  done
done
