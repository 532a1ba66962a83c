#!/usr/bin/env bash
# Round-5 GPU batch 13: the proof launches reading f * h^2 (B_FH) - parity
# tests of the red-black cavity paths, then the headline bench three times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b13; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_proof.py tests/test_gpu_pairs.py tests/test_gpu_ranks.py tests/test_gpu_baseline_configs.py -m gpu > $D/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -n 3 $D/pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $D/pytest.log | head; exit $rc; }
for i in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --lex-steps 0 > $D/bench$i.json 2>> $D/err.log || exit $?
  python3 -c "import json;d=json.load(open('$D/bench$i.json'));print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'],d['roofline']['frac'])"
done
