#!/usr/bin/env bash
# One-step bench lines over a launch-plan knob (performance only: every value
# gives the same bits). SWEEP="name:bench args:knob:v1 v2 ..;..." -> $D/<name>_<knob><v>.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${OUT:-gpurun_out/tune}; mkdir -p $D
IFS=';' read -ra WL <<< "$SWEEP"
for w in "${WL[@]}"; do
  IFS=: read -r n a knob vals <<< "$w"
  for v in $vals; do
    timeout -k 10 200 python3 bench.py $a --steps ${STEPS:-1} --warmup 1 --no-cpu-baseline --lex-steps 0 --tune $knob=$v > $D/${n}_$knob$v.json 2> $D/${n}_$knob$v.err || exit 1
    python3 -c "import json;d=json.load(open('$D/${n}_$knob$v.json'));print('$n', '$knob', $v, round(d['value']/1e3,1), d['ms_per_step'], d['roofline']['avg_launch_us'])"
  done
done
