set -o pipefail
# chunked-sum tests, phase stamps (diagnostic build) and the kernel trace of
# the open cases' reference-order benches -> gpurun_out/seqsum/
D=gpurun_out/seqsum; mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_seqsum.py > $D/t_seqsum.log 2>&1 || { tail -40 $D/t_seqsum.log; exit 1; }
tail -1 $D/t_seqsum.log
CFD_AMD_LIB=libcfd_amd_sstamps.so timeout -k 10 200 python -u scripts/dbg/seqsum_stamps.py > $D/stamps.log 2>&1 || { tail $D/stamps.log; exit 1; }
cat $D/stamps.log
bash scripts/dbg/seqsum_prof.sh 2>&1 | grep -v t_seqsum
