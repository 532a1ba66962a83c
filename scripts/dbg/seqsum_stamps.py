"""Phase times of seq_walk_kernel (diagnostic build: make variant NAME=sstamps
DEFS=-DCFD_SEQ_STAMPS=1; run with CFD_AMD_LIB=libcfd_amd_sstamps.so)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "computational-fluid-dynamics_amd"))
import cfd_amd as C  # noqa: E402
from cfd_amd import _lib  # noqa: E402

L = _lib.lib()
L.cfd_seq_stamps.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
names = ["batch loads", "run records", "single records", "staging", "plain chains"]
for case, kw in {"channel": dict(nx=4096, ny=512, re=1000), "backwards_step": dict(nx=8192, ny=512, re=400)}.items():
    cp = C.make_params(case, **kw)
    g = {"channel": C.ChannelSolver, "backwards_step": C.BackwardsStepSolver}[case](cp, ordering="lex")
    for s in range(3):
        g.reset_timing()
        g.step()
        t = g.timing()
        out = (ctypes.c_int * 5)()
        L.cfd_seq_stamps(g._h, out)
        print(case, "step", s + 1, "chunks", t.seqsum_chunks, "plain", t.seqsum_serial_chunks,
              {n: round(v / 100.0, 1) for n, v in zip(names, out)}, "(us)", flush=True)
