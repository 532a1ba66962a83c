#!/usr/bin/env bash
# Copy the round evidence of scripts/profile_case.sh runs (gpurun_out/prof/<TAG>/)
# into profiles/ as r<ROUND>_bench_<TAG>.json, r<ROUND>_kernel_stats_<TAG>.csv and
# r<ROUND>_pmc_<TAG>.json (the PMC file carries the kernel's source hash:
# bench.py reports its traffic only while the sources match).
#   ROUND=6 bash scripts/collect_profiles.sh [TAG ...]   (default: every TAG present)
set -e
cd "$(dirname "$0")/.."
R=${ROUND:?ROUND= required}
tags=("$@")
[ ${#tags[@]} -eq 0 ] && tags=($(ls gpurun_out/prof))
for t in "${tags[@]}"; do
  d=gpurun_out/prof/$t
  [ -s $d/bench.json ] && cp $d/bench.json profiles/r${R}_bench_$t.json && echo "profiles/r${R}_bench_$t.json"
  f=$(find $d/stats -name '*kernel_stats.csv' 2>/dev/null | head -1)
  [ -n "$f" ] && cp "$f" profiles/r${R}_kernel_stats_$t.csv && echo "profiles/r${R}_kernel_stats_$t.csv"
  [ -s $d/pmc.json ] && cp $d/pmc.json profiles/r${R}_pmc_$t.json && echo "profiles/r${R}_pmc_$t.json"
done
