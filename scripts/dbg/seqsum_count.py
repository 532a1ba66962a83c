"""Chunks / plain-chain chunks of the sequential source sums over a few
reference-order steps of the open cases' bench configurations."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "computational-fluid-dynamics_amd"))
import cfd_amd as C  # noqa: E402

for case, kw in {"channel": dict(nx=4096, ny=512, re=1000), "backwards_step": dict(nx=8192, ny=512, re=400)}.items():
    cp = C.make_params(case, **kw)
    g = {"channel": C.ChannelSolver, "backwards_step": C.BackwardsStepSolver}[case](cp, ordering="lex")
    for s in range(4):
        g.reset_timing()
        g.step()
        t = g.timing()
        print(case, "step", s + 1, "chunks", t.seqsum_chunks, "plain", t.seqsum_serial_chunks, flush=True)
