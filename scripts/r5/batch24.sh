#!/usr/bin/env bash
# Round-5 GPU batch 24: wholly active wall tiles of the reference order's ramp
# launches on the unmasked edge march - lexw tests and digests, then the step
# and cavity 4096^2 reference-order benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b26; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_lexw.py tests/test_gpu_lex_digests.py tests/test_gpu_lex.py > $D/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -n 2 $D/pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $D/pytest.log | head; exit $rc; }
timeout -k 10 300 python3 -u bench.py --case backwards_step --nx 8192 --ny 512 --re 400 --ordering lex --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0 > $D/step.json 2>> $D/err.log || exit $?
python3 -c "import json;d=json.load(open('$D/step.json'));print('step lex',d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'])"
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --ordering lex --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0 > $D/cav$i.json 2>> $D/err.log || exit $?
python3 -c "import json;d=json.load(open('$D/cav$i.json'));print('cavity lex 4096',d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'])"
done
