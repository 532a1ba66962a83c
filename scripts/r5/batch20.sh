#!/usr/bin/env bash
# Round-5 GPU batch 20: the step's ramp band floor default (100) - the step's
# reference-order tests and digests, then its bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b20; mkdir -p $D
timeout -k 10 700 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_lexw.py tests/test_gpu_lex_digests.py tests/test_gpu_smlex.py -k "step or digest" > $D/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -n 2 $D/pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $D/pytest.log | head; exit $rc; }
timeout -k 10 300 python3 -u bench.py --case backwards_step --nx 8192 --ny 512 --re 400 --ordering lex --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0 > $D/bench_step_lex.json 2>> $D/err.log || exit $?
python3 -c "import json;d=json.load(open('$D/bench_step_lex.json'));print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'])"
