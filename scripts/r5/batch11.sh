#!/usr/bin/env bash
# Round-5 GPU batch 11: the whole GPU suite with the channel's resident
# default, then the step's reference-order launch stamps after the splits.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b11; mkdir -p $D
timeout -k 10 1000 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -n 5 $D/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $D/pytest_gpu.log | head; exit $rc; }
CFD_AMD_LIB=$PWD/computational-fluid-dynamics_amd/libcfd_amd_lstamps.so timeout -k 10 240 python3 -u scripts/dbg/lexw_stamps.py backwards_step 8192 512 > $D/step_stamps.json 2> $D/step_stamps.err || exit $?
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r5b11/step_stamps.json"))
for t in d["by_tenth"]:
    print(t["launches"], t["launch_max_cycles_mean"], t["slowest_path"], {k: (round(v["waves_per_launch"]), v["max_cycles_mean"]) for k, v in t["paths"].items()})
PY
