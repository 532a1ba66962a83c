#!/usr/bin/env bash
# Round-5 GPU batch 12: the reference order at 4096^2 - 4 vs 5 sweeps per
# launch, and the ramp band floor (lexw_ramp_pct) - A/B on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
D=gpurun_out/r5b12; mkdir -p $D
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --lex-steps 0 > $D/rb_headline.json 2>> $D/err.log || exit $?
python3 -c "import json;d=json.load(open('$D/rb_headline.json'));print('rb headline',d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'])"
for spl in 4 5 4 5; do
  timeout -k 10 300 python3 -u bench.py --ordering lex --sweeps-per-launch $spl --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0 > $D/lex_spl$spl.json 2>> $D/err.log || exit $?
  python3 -c "import json;d=json.load(open('$D/lex_spl$spl.json'));print('spl',$spl,d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'])"
done
for rp in 0 50 100; do
  timeout -k 10 300 python3 -u bench.py --ordering lex --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0 --tune lexw_ramp_pct=$rp > $D/lex_rp$rp.json 2>> $D/err.log || exit $?
  python3 -c "import json;d=json.load(open('$D/lex_rp$rp.json'));print('ramp_pct',$rp,d['value'],d['ms_per_step'])"
done
