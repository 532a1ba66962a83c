"""Host restatement of seqsum.hip's binade-chunked sequential sum, checked bit
for bit against the plain chain (one IEEE rounding per term, the reference's
loop: channel-01.cpp:620-628, backwards_step-01.cpp:843-866) on terms built to
stress it: the open cases' shape (a steady mean plus noise), random signs over
many binades (the running sum crossing zero), exact ties at the running sum's
unit, -0.0 solids, a carried start (strips / ranks), non-finite terms. It pins
the integer-path argument on the CPU; tests/test_gpu_seqsum.py runs the kernels
themselves against the same plain chain."""
from __future__ import annotations

import math

import numpy as np
import pytest

CH = 512           # SQ_CH
L_, H_ = 2 ** 52 + 1, 2 ** 53 - 1


def chain(x, s=0.0):
    for v in x.tolist():
        s = s + v
    return s


def chunk_record(block, u):
    """seq_chunk_kernel: per incoming parity (R, min, max) of the integer prefix sums, or None (serial)."""
    y = np.ldexp(block, -u)
    if not np.all(np.abs(y) < 2.0 ** 51):
        return None
    tr = np.trunc(y)
    fr = y - tr
    tie = np.abs(fr) == 0.5
    r = tr.astype(np.int64) + (fr > 0.5) - (fr < -0.5)
    q = np.floor(y).astype(np.int64)
    recs = []
    for par in (0, 1):
        if not tie.any():
            p = np.cumsum(r)
            recs.append((int(p[-1]), min(0, int(p.min())), max(0, int(p.max()))))
            continue
        R = lo = hi = 0
        for k in range(block.size):
            R += int(q[k]) + ((par + R + int(q[k])) & 1) if tie[k] else int(r[k])
            lo, hi = min(lo, R), max(hi, R)
        recs.append((R, lo, hi))
    return recs


def combine(a, b):
    """meta_combine: a then b, b's record chosen by the parity a hands over."""
    out = []
    for p in (0, 1):
        R, lo, hi = a[p]
        bR, blo, bhi = b[(p + R) & 1]
        out.append((R + bR, min(lo, R + blo), max(hi, R + bhi)))
    return out


def apply(s, recs, u):
    """meta_apply: the exact check, then s + the record by the integer path."""
    if recs is None:
        return None
    S = math.ldexp(s, -u) if math.isfinite(s) else math.inf
    if not (2.0 ** 52 <= abs(S) < 2.0 ** 53):
        return None
    Si = int(S)
    R, lo, hi = recs[Si & 1]
    ok = (Si + lo >= L_ and Si + hi <= H_) if Si > 0 else (Si + hi <= -L_ and Si + lo >= -H_)
    return math.ldexp(float(Si + R), u) if ok else None


def chunked(x, s0=0.0):
    """seq_approx/units/chunk kernels + seq_walk_kernel (the longest passing prefix of up to 64 chunks)."""
    nch = (x.size + CH - 1) // CH
    blocks = np.concatenate([x, np.full(nch * CH - x.size, -0.0)]).reshape(nch, CH)
    with np.errstate(invalid="ignore", over="ignore"):
        approx = blocks.sum(axis=1)
        pre = np.concatenate([[0.0], np.cumsum(approx)[:-1]]) + s0
    units = [math.frexp(p)[1] - 53 if math.isfinite(p) else 0 for p in pre]
    recs = [chunk_record(blocks[c], units[c]) for c in range(nch)]
    s, k, plain = s0, 0, 0
    while k < nch:
        run = 0
        while run < 64 and k + run < nch and units[k + run] == units[k]:
            run += 1
        acc, take, s_new = None, 0, None
        for c in range(k, k + run):
            if recs[c] is None:
                break
            acc = recs[c] if acc is None else combine(acc, recs[c])
            t = apply(s, acc, units[k])
            if t is None:
                break
            take, s_new = take + 1, t
        if take:
            s, k = s_new, k + take
            continue
        plain += 1
        s, k = chain(blocks[k], s), k + 1
    return s, nch, plain


def same_bits(a, b):
    return np.float64(a).view(np.int64) == np.float64(b).view(np.int64) or (math.isnan(a) and math.isnan(b))


def _terms(kind, rng, n):
    if kind == "drift":
        return -9900.0 + rng.normal(0.0, 50.0, n)
    if kind == "signs":
        return rng.choice([-1.0, 1.0], n) * np.exp(rng.normal(0.0, 8.0, n))
    if kind == "ties":
        return 1024.0 * rng.integers(2 ** 39, 2 ** 41, n).astype(np.float64)
    if kind == "halves":
        return rng.integers(1, 2 ** 20, n) + 0.5
    if kind == "solids":
        return np.where(rng.random(n) < 0.3, -0.0, rng.normal(-5.0, 1.0, n))
    raise ValueError(kind)


@pytest.mark.parametrize("kind,s0", [("drift", 0.0), ("signs", 0.0), ("ties", 0.0), ("halves", 2.0 ** 52),
                                     ("solids", 0.0), ("drift", -1.0e6), ("signs", 3.5e12)])
def test_chunked_equals_plain_chain(kind, s0):
    rng = np.random.default_rng([len(kind), ord(kind[0]), int(abs(s0)) % 100003])
    x = _terms(kind, rng, 150_000)
    want = chain(x, s0)
    got, nch, plain = chunked(x, s0)
    assert same_bits(want, got), (want, got)
    if kind in ("drift", "ties", "halves", "solids"):
        assert plain <= nch // 4, (plain, nch)


def test_chunked_non_finite_and_empty():
    x = np.full(10_000, 1.25)
    x[3000], x[7000] = np.inf, -np.inf
    got, _, _ = chunked(x)
    assert math.isnan(got) and math.isnan(chain(x))
    assert chunked(np.zeros(0), 2.5)[0] == 2.5
