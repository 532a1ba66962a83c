set -o pipefail
export CFD_COMMIT=$1
bash scripts/seqsum_ranks.sh > gpurun_out/seqsum_ranks.log 2>&1 || { tail gpurun_out/seqsum_ranks.log; exit 1; }
cat gpurun_out/seqsum_ranks.log
bash scripts/profile_round.sh > gpurun_out/profile_round.log 2>&1
rc=$?; grep -E "exit|hbm_bytes|traffic_over|pmc ok" gpurun_out/profile_round.log | head -60; exit $rc
