set -o pipefail
export CFD_COMMIT=d526f0d
CFD_AMD_LIB=libcfd_amd_lstamps.so timeout -k 10 120 python3 -u scripts/dbg/lexw_stamps.py cavity 4096 4096 10000 > gpurun_out/r6_stamps_cav4k_lex.json 2> gpurun_out/r6_stamps.err || { tail gpurun_out/r6_stamps.err; exit 1; }
CASES=cav4klex bash scripts/profile_round.sh
