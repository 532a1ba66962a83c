set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lexw.py -k "five or step" > gpurun_out/ab5_tests.log 2>&1 || { tail -30 gpurun_out/ab5_tests.log; exit 1; }
tail -2 gpurun_out/ab5_tests.log
timeout -k 10 300 python3 -u - <<'PY' || exit 1
import sys, json, hashlib, numpy as np
sys.path.insert(0, "computational-fluid-dynamics_amd")
import cfd_amd as C
d = json.load(open("tests/golden/lex_digests.json"))["backwards_step_8192x512_K4400"]
kw = dict(d["params"]); kw.pop("case")
cp = C.make_params("backwards_step", **kw)
g = C.BackwardsStepSolver(cp, ordering="lex", small_solve="off", sweeps_per_launch=5)
it, res = g.step()
dig = {n: hashlib.sha256(np.ascontiguousarray(g.field(n), dtype="<f8").tobytes()).hexdigest() for n in ("u", "v", "p")}
print("digest 5 sweeps", it == d["sor_iterations"], res.hex() == d["residual"], dig == d["sha256"], g.timing().poisson_steady_launches)
PY
for v in 5 0 5 0; do
  timeout -k 10 200 python -u bench.py --case backwards_step --nx 8192 --ny 512 --re 400 --steps 2 --warmup 1 --no-cpu-baseline --lex-steps 0 --sweeps-per-launch $v > gpurun_out/ab5_b$v.json 2> gpurun_out/ab5_b$v.err || { tail gpurun_out/ab5_b$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab5_b$v.json')); r=d['roofline']; print('step spl=$v', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'])"
done
