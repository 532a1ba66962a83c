"""CPU emulation of seqsum.hip's binade-chunked sequential sum against the
plain chain, on the open cases' dumped sources (scripts/dbg/dump_src.py ->
gpurun_out/src_<case>.npz) and on adversarial terms (sign changes, wide
magnitudes, ties). Prints chunks, plain-chain chunks and whether the bits
agree. Host-only: python scripts/dbg/seqsum_study.py"""
import math
import os
import sys

import numpy as np

CH = 512  # SQ_CH


def chain(x, s=0.0):
    for v in x.tolist():
        s = s + v
    return s


def chunked(x, s0=0.0):
    n = x.size
    nch = (n + CH - 1) // CH
    xp = np.concatenate([x, np.full(nch * CH - n, -0.0)])
    blocks = xp.reshape(nch, CH)
    approx = blocks.sum(axis=1)
    pre = np.concatenate([[0.0], np.cumsum(approx)[:-1]]) + s0
    metas = []
    for c in range(nch):
        e = math.frexp(pre[c])[1]
        u = e - 53
        y = np.ldexp(blocks[c], -u)
        if not np.all(np.abs(y) < 2.0 ** 51):
            metas.append((None, u, True))
            continue
        tr = np.trunc(y)
        fr = y - tr
        tie = np.abs(fr) == 0.5
        r = tr.astype(np.int64) + (fr > 0.5) - (fr < -0.5)
        if not tie.any():
            p = np.cumsum(r)
            rec = (int(p[-1]), min(0, int(p.min())), max(0, int(p.max())))
            metas.append(((rec, rec), u, False))
            continue
        # ties: one record per parity of the incoming integer sum (the even
        # neighbour of S + q is taken: r = q + ((S + q) & 1))
        q = np.floor(y).astype(np.int64)
        recs = []
        for par in (0, 1):
            R, lo, hi = 0, 0, 0
            for k in range(CH):
                rk = int(q[k]) + ((par + R + int(q[k])) & 1) if tie[k] else int(r[k])
                R += rk
                lo, hi = min(lo, R), max(hi, R)
            recs.append((R, lo, hi))
        metas.append((tuple(recs), u, False))
    s = s0
    nser = 0
    L, H = 2 ** 52 + 1, 2 ** 53 - 1
    for c, (recs, u, serial) in enumerate(metas):
        ok = False
        if not serial:
            S = math.ldexp(s, -u)
            if 2.0 ** 52 <= abs(S) < 2.0 ** 53:
                Si = int(S)
                R, lo, hi = recs[Si & 1]
                a, b = Si + lo, Si + hi
                ok = (a >= L and b <= H) if Si > 0 else (b <= -L and a >= -H)
                if ok:
                    s = math.ldexp(float(Si + R), u)
        if not ok:
            nser += 1
            s = chain(blocks[c], s)
    return s, nch, nser


def check(name, x, s0=0.0):
    want = chain(x, s0)
    got, nch, nser = chunked(x, s0)
    same = (np.float64(want).view(np.int64) == np.float64(got).view(np.int64))
    print(f"{name}: {nch} chunks, {nser} plain, bits equal {bool(same)} ({want!r} vs {got!r})", flush=True)
    return same


if __name__ == "__main__":
    rng = np.random.default_rng(7)
    ok = True
    for case in ("channel", "backwards_step"):
        path = os.path.join("gpurun_out", f"src_{case}.npz")
        if os.path.exists(path):
            d = np.load(path)
            for k in d.files:
                if k.startswith("f"):
                    ok &= check(f"{case} {k}", d[k].ravel())
    n = 300_000
    ok &= check("random signs, lognormal", rng.choice([-1.0, 1.0], n) * np.exp(rng.normal(0, 8, n)))
    ok &= check("drift + noise", -9900.0 + rng.normal(0, 50, n))
    ok &= check("ties (integers x 1024 past 2^63)", 1024.0 * rng.integers(2 ** 39, 2 ** 41, n).astype(np.float64))
    ok &= check("half-integers past 2^52", rng.integers(1, 2 ** 20, n) + 0.5, s0=2.0 ** 52)
    ok &= check("from a carried start", rng.normal(3.0, 1.0, n), s0=-1.0e6)
    ok &= check("with -0.0 solids", np.where(rng.random(n) < 0.3, -0.0, rng.normal(-5.0, 1.0, n)))
    sys.exit(0 if ok else 1)
