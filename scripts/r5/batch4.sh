#!/usr/bin/env bash
# Round-5 GPU batch 4: resident solve - phase stamps (diagnostic build), the
# product's bit tests and solve times vs the LDS tiles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b4; mkdir -p $D
for g in "1024 1024" "1024 64"; do
  CFD_AMD_LIB=libcfd_amd_rstamps.so timeout -k 10 120 python3 -u scripts/dbg/res_stamps.py $g 2000 >> $D/stamps.txt 2>&1 || exit 1
done
python3 -c "
import json,re
t=open('$D/stamps.txt').read()
for blk in re.findall(r'\{.*?\}', t, re.S):
    d=json.loads(blk); print(d['nx'],d['ny'],'us/sweep',round(d['us_per_sweep'],3),{k.replace('_cyc_per_group',''):v for k,v in d.items() if 'cyc' in k})"
timeout -k 10 300 python3 -u scripts/r5/resdbg.py > $D/resdbg.txt 2>&1; rc=$?; cat $D/resdbg.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_resident.py > $D/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -n 3 $D/pytest.log; exit $rc
