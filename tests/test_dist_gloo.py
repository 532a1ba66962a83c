"""World-size-2 gloo tests of the multi-process strip decomposition (CPU).

The GPU data path (RCCL send/recv of halo rows inside libcfd_amd.so) needs
GPUs; here we check the host logic around it and the decomposition itself:
row partitioning, RCCL-id bootstrap over a process group, max-over-ranks
timing, and a numpy emulation of the fused red-black SOR launches on two
strips: HALO=8 rows exchanged over gloo, then two or three iterations computed locally
(the GPU's multi-iteration kernel, poisson_multi_kernel: 2, or 3 for the
cavity), a shorter last launch for the remainder. It must equal the single-domain iteration bit for bit, both
residuals included (the property the GPU kernels rely on: redundant
recomputation of the halo rows reproduces the neighbour's arithmetic).
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from cfd_amd.dist import HALO, broadcast_comm_id, max_over_ranks, strip_rows, sum_over_ranks, weak_rows


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_strip_rows_partition():
    for ny, world in [(4096, 8), (63, 2), (1000, 3), (32, 4)]:
        rows = [strip_rows(r, world, ny) for r in range(world)]
        assert rows[0][0] == 1 and rows[-1][1] == ny
        for (a0, a1), (b0, b1) in zip(rows, rows[1:]):
            assert b0 == a1 + 1
        assert max(b - a for a, b in rows) - min(b - a for a, b in rows) <= 1
    with pytest.raises(ValueError):
        strip_rows(0, 16, 40)
    assert weak_rows(3, 4096) == (12289, 16384)


# ---- numpy restatement of one cavity red-black SOR iteration (csrc/kernels.hpp) ----

def rb_iteration(p, f, nx, ny, omega, h, j_lo, j_hi):
    """One red-black sweep on rows [j_lo, j_hi] of the arrays (global row index
    j -> array row j - j_lo + HALO... caller passes arrays already offset) and
    the max residual over the rows given."""
    p = p.copy()
    jj, ii = np.meshgrid(np.arange(p.shape[0]) + j_lo, np.arange(p.shape[1]), indexing="ij")
    inside = (ii >= 1) & (ii <= nx) & (jj >= 1) & (jj <= ny)
    for color in (0, 1):
        m = inside & (((ii + jj) & 1) == color)
        m[0, :] = m[-1, :] = False  # need both vertical neighbours stored
        ee = (ii < nx).astype(float); ew = (ii > 1).astype(float); en = (jj < ny).astype(float)
        nc = ee + ew + en + 1.0
        pE = np.roll(p, -1, 1); pW = np.roll(p, 1, 1); pN = np.roll(p, -1, 0); pS = np.roll(p, 1, 0)
        new = p * (1.0 - omega) + (omega / nc) * ((ee * pE + ew * pW) + (en * pN + pS) - f * (h * h))
        p = np.where(m, new, p)
    return p


def residual(p, f, nx, ny, h, j_lo):
    jj, ii = np.meshgrid(np.arange(p.shape[0]) + j_lo, np.arange(p.shape[1]), indexing="ij")
    ee = (ii < nx).astype(float); ew = (ii > 1).astype(float); en = (jj < ny).astype(float)
    c = p
    r = (1.0 / (h * h)) * (ee * (np.roll(p, -1, 1) - c) + ew * (np.roll(p, 1, 1) - c) + en * (np.roll(p, -1, 0) - c)
                           + (np.roll(p, 1, 0) - c)) - f
    inside = (ii >= 1) & (ii <= nx) & (jj >= 1) & (jj <= ny)
    inside[0, :] = inside[-1, :] = False
    return np.where(inside, np.abs(r), 0.0)


def _worker(rank, world, port, q, nx, ny, iters, spl):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    try:
        # bootstrap: rank 0's id reaches everyone
        cid = broadcast_comm_id(dist, rank, lambda: bytes(range(128)))
        assert cid == bytes(range(128))
        # timing reductions
        assert max_over_ranks(dist, float(rank + 1)) == float(world)
        assert sum_over_ranks(dist, 1.0) == float(world)
        # strip-decomposed red-black SOR with HALO-row exchange
        rng = np.random.default_rng(0)
        f_full = np.zeros((ny + 2, nx + 2)); f_full[1:ny + 1, 1:nx + 1] = rng.standard_normal((ny, nx))
        h, omega = 1.0 / nx, 1.7
        j0, j1 = strip_rows(rank, world, ny)
        lo = j0 - HALO  # global row of local row 0
        rows = np.arange(lo, j1 + HALO + 1)
        valid = (rows >= 0) & (rows <= ny + 1)
        f = np.zeros((len(rows), nx + 2)); f[valid] = f_full[rows[valid]]
        p = np.zeros_like(f)
        res_hist = []
        done = 0
        while done < iters:
            n = min(spl, iters - done)  # iterations fused into this launch
            # exchange HALO owned rows with the neighbours (the GPU path: ncclSend/ncclRecv)
            if rank > 0:
                dist.send(torch.from_numpy(p[HALO:2 * HALO].copy()), rank - 1)
                buf = torch.empty((HALO, nx + 2), dtype=torch.float64); dist.recv(buf, rank - 1)
                p[:HALO] = buf.numpy()
            if rank < world - 1:
                buf = torch.empty((HALO, nx + 2), dtype=torch.float64); dist.recv(buf, rank + 1)
                top = p[-2 * HALO:-HALO].copy()
                dist.send(torch.from_numpy(top), rank + 1)
                p[-HALO:] = buf.numpy()
            pn = p
            for _ in range(n):  # halo rows recomputed redundantly, no exchange in between
                pn = rb_iteration(pn, f, nx, ny, omega, h, lo, None)
                r = residual(pn, f, nx, ny, h, lo)[HALO:-HALO].max()
                res_hist.append(max_over_ranks(dist, r))
            done += n
            # keep owned rows (halo rows are refreshed by the next exchange)
            p[HALO:-HALO] = pn[HALO:-HALO]
            if rank == 0:
                p[:HALO] = pn[:HALO]  # physical ghost rows live in the first strip's halo
            if rank == world - 1:
                p[-HALO:] = pn[-HALO:]
        q.put((rank, j0, j1, p[HALO:-HALO].copy(), res_hist))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("spl", [2, 3])
@pytest.mark.parametrize("world,nx,ny", [(2, 24, 20), (2, 40, 1024)])
def test_two_rank_strips_equal_single_domain(world, nx, ny, spl):
    """(2, 40, 1024): 512 rows per rank, the strip height of the strong-scaling
    bench (4096² over 8 GPUs)."""
    iters = 15
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, nx, ny, iters, spl)) for r in range(world)]
    for pr in procs:
        pr.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    # single domain
    rng = np.random.default_rng(0)
    f = np.zeros((ny + 2, nx + 2)); f[1:ny + 1, 1:nx + 1] = rng.standard_normal((ny, nx))
    p = np.zeros_like(f)
    hist = []
    for _ in range(iters):
        p = rb_iteration(np.vstack([p]), f, nx, ny, 1.7, 1.0 / nx, 0, None)
        hist.append(residual(p, f, nx, ny, 1.0 / nx, 0).max())
    for rank, j0, j1, strip, res_hist in out:
        assert np.array_equal(strip, p[j0:j1 + 1])
        assert res_hist == hist


# ---- the default rank launch: 4 sweeps with the proof-mode test ----

def proof_ratio(dmax, pin, F, tol, h, omega, ns):
    """kernels.hpp proof_ratio (the launch kernel's form, P bounded per rank)."""
    idx2 = 1.0 / (h * h)
    K = 4.0 * idx2 * abs(1.0 - omega) / omega
    P = 9.0**ns * (pin + h * h * F) * (1.0 + 2.0**-40)
    margin = 2.0**-43 * (idx2 * P + F)
    thr = (tol + margin) / K * (1.0 + 2.0**-38)
    q = dmax / thr
    return q if (q == q and q >= 0.0) else 0.0


def black_moves(p_old, p_new, nx, ny, lo):
    """max |p' - p| over the black four-neighbour cells (1 < i < nx, 1 <= j < ny)."""
    jj, ii = np.meshgrid(np.arange(p_old.shape[0]) + lo, np.arange(p_old.shape[1]), indexing="ij")
    m = (ii > 1) & (ii < nx) & (jj >= 1) & (jj < ny) & (((ii + jj) & 1) == 1)
    m[0, :] = m[-1, :] = False
    return float(np.abs(np.where(m, p_new - p_old, 0.0)).max())


def _solve_ranks(rank, world, nx, ny, f_full, omega, tol, cap, chunk, exchange, allmax):
    """Solver::solve on one rank: launches of 4 proof-mode sweeps, the window of
    each launch tested after it (all-reduced ratio > 1: proven); an iteration
    the proof leaves open restarts the solve at that launch with exact 3-sweep
    launches (all-reduced max-norm residual <= tol: the reference stops) for
    `chunk` launches, then proof mode again. Returns the owned rows, the stop
    iteration and the launch indices of the fallbacks."""
    h = 1.0 / nx
    j0, j1 = strip_rows(rank, world, ny)
    lo = j0 - HALO
    rows = np.arange(lo, j1 + HALO + 1)
    valid = (rows >= 0) & (rows <= ny + 1)
    f = np.zeros((len(rows), nx + 2)); f[valid] = f_full[rows[valid]]
    F = float(np.abs(f_full[1:ny + 1, 1:nx + 1]).max())
    p = np.zeros_like(f)
    k, m, proof_from, fallbacks = 0, 0, 0, []
    alone = 0  # sweeps this rank alone could not prove but the all-reduced ratio did
    while k < cap:
        proof = m >= proof_from
        n = min(4 if proof else 3, cap - k)
        exchange(p)
        pin = float(np.abs(p).max())
        pn, stop, open_k = p, None, None
        for s in range(n):
            prev = pn
            pn = rb_iteration(pn, f, nx, ny, omega, h, lo, None)
            if proof and n >= 3:
                ql = proof_ratio(black_moves(prev, pn, nx, ny, lo), pin, F, tol, h, omega, n)
                q = allmax(ql)
                alone += int(not ql > 1.0 and q > 1.0)
                if not q > 1.0 and open_k is None:
                    open_k = k + s + 1
            else:
                r = allmax(residual(pn, f, nx, ny, h, lo)[HALO:-HALO].max())
                if not r > tol and stop is None and open_k is None:
                    stop = k + s + 1
                    pstop = pn.copy()
        if open_k is not None:  # exact evaluation from this launch's (intact) input
            fallbacks.append(m)
            proof_from = m + chunk
            continue  # same m, same k, now exact (p is this launch's input: nothing was written)
        if stop is not None:
            pn = pstop
            k = stop
            p[HALO:-HALO] = pn[HALO:-HALO]
            break
        k += n
        m += 1
        p[HALO:-HALO] = pn[HALO:-HALO]
        if rank == 0:
            p[:HALO] = pn[:HALO]
        if rank == world - 1:
            p[-HALO:] = pn[-HALO:]
    return j0, j1, p[HALO:-HALO].copy(), k, fallbacks, alone


def _proof_worker(rank, world, port, q, nx, ny, tol, cap, chunk):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    try:
        def exchange(p):
            if rank > 0:
                dist.send(torch.from_numpy(p[HALO:2 * HALO].copy()), rank - 1)
                buf = torch.empty((HALO, p.shape[1]), dtype=torch.float64); dist.recv(buf, rank - 1)
                p[:HALO] = buf.numpy()
            if rank < world - 1:
                buf = torch.empty((HALO, p.shape[1]), dtype=torch.float64); dist.recv(buf, rank + 1)
                dist.send(torch.from_numpy(p[-2 * HALO:-HALO].copy()), rank + 1)
                p[-HALO:] = buf.numpy()

        q.put((rank,) + _solve_ranks(rank, world, nx, ny, _proof_source(nx, ny), 1.8, tol, cap, chunk, exchange,
                                     lambda v: max_over_ranks(dist, v)))
    finally:
        dist.destroy_process_group()


def _proof_source(nx, ny):
    """A source on the upper rank's rows only: the lower rank's own black moves
    stay far below the threshold for the first launches, so a rank deciding
    alone would fall back there; the all-reduced ratio decides for both."""
    rng = np.random.default_rng(3)
    f = np.zeros((ny + 2, nx + 2))
    f[ny // 2 + 4:ny + 1, 1:nx + 1] = rng.standard_normal((ny - ny // 2 - 3, nx)) * 50.0
    return f


@pytest.mark.parametrize("tol,cap", [(20.0, 400), (12.0, 400), (1e9, 400), (0.0, 37)])
def test_two_rank_proof_launches_equal_single_domain(tol, cap):
    """Two gloo ranks of 64 rows (the same 8-row halos as the GPU's 512-row
    strips): the 4-sweep proof-mode launch, ratios
    all-reduced (max) like the GPU's ring slots, a fallback taken by both ranks
    at the same launch, exact launches for a chunk, proof again. The stop
    iteration and the fields must equal one domain with an exact residual test
    every sweep (the reference's loop in red-black order); a capped solve never
    falls back after its first launches."""
    world, nx, ny, chunk = 2, 40, 128, 2
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_proof_worker, args=(r, world, port, qq, nx, ny, tol, cap, chunk))
             for r in range(world)]
    for pr in procs:
        pr.start()
    out = sorted(qq.get(timeout=300) for _ in range(world))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    # one domain, exact residual after every sweep
    f = _proof_source(nx, ny)
    p = np.zeros_like(f)
    k = 0
    while k < cap:
        p = rb_iteration(p, f, nx, ny, 1.8, 1.0 / nx, 0, None)
        k += 1
        if not residual(p, f, nx, ny, 1.0 / nx, 0).max() > tol:
            break
    fb = [o[5] for o in out]
    assert fb[0] == fb[1], "both ranks fall back at the same launches"
    for rank, j0, j1, strip, kk, _, _ in out:
        assert kk == k
        assert np.array_equal(strip, p[j0:j1 + 1])
    if tol == 1e9:
        assert k == 1  # (the first iteration already meets it)
    if 0.0 < tol < 1e9:
        assert len(fb[0]) >= 1  # converging: the last iterations are evaluated exactly
        assert out[0][6] > 0  # the lower rank alone would have fallen back earlier


# ---- the reference's order on ranks (Solver::solve_lexw with a communicator) ----
#
# The lexicographic sweep (cavity-01.cpp:640-656) as the skewed half-sweep
# schedule the GPU runs (csrc/lexw.hpp: cell (j, i) performs its iteration k
# at half-sweep i + j + 2(k - 1)), on two gloo ranks: HALO rows exchanged
# before every launch of 3 sweeps (6 half-sweeps, the halo rows recomputed
# redundantly), each cell's iteration-k residual evaluated in the half-sweep
# after its update (W, S before it, E, N after: the reference's operands), one
# exceedance bit per iteration per rank, OR-ed over the ranks with a max
# all-reduce (Solver::lexw_reduce_bits), the stop at the first iteration
# without one and the replay of that many iterations from the initial field.
# Must equal the reference's loop on one domain bit for bit: fields, stop.

LEX_NS = 3


def _lex_formula(c, pE, pW, pN, pS, f, ee, ew, en, omega, h):
    nc = ee + ew + en + 1.0
    return c * (1.0 - omega) + (omega / nc) * ((ee * pE + ew * pW) + (en * pN + pS) - f * (h * h))


def _lex_res(c, pE, pW, pN, pS, f, ee, ew, en, h):
    return (1.0 / (h * h)) * (ee * (pE - c) + ew * (pW - c) + en * (pN - c) + (pS - c)) - f


def lex_reference(f, nx, ny, omega, h, K, tol):
    """The reference's loop (scalar Python, one domain): sweep j = 1..ny,
    i = 1..nx in place, then the max-norm residual; stop when it is <= tol."""
    p = np.zeros_like(f)
    for k in range(1, K + 1):
        for j in range(1, ny + 1):
            for i in range(1, nx + 1):
                ee, ew, en = float(i < nx), float(i > 1), float(j < ny)
                p[j, i] = _lex_formula(p[j, i], p[j, i + 1], p[j, i - 1], p[j + 1, i], p[j - 1, i], f[j, i],
                                       ee, ew, en, omega, h)
        r = 0.0
        for j in range(1, ny + 1):
            for i in range(1, nx + 1):
                ee, ew, en = float(i < nx), float(i > 1), float(j < ny)
                r = max(r, abs(_lex_res(p[j, i], p[j, i + 1], p[j, i - 1], p[j + 1, i], p[j - 1, i], f[j, i],
                                        ee, ew, en, h)))
        if not r > tol:
            return p, k
    return p, K


def _lex_skewed(rank, world, nx, ny, f_full, omega, h, K, tol, exchange, ormax):
    """One rank's skewed solve of K iterations; returns its owned rows and the
    iteration the (all-reduced) bits stop at (K: none)."""
    j0, j1 = strip_rows(rank, world, ny)
    lo = j0 - HALO
    rows = np.arange(lo, j1 + HALO + 1)
    valid = (rows >= 0) & (rows <= ny + 1)
    f = np.zeros((len(rows), nx + 2)); f[valid] = f_full[rows[valid]]
    jj, ii = np.meshgrid(rows, np.arange(nx + 2), indexing="ij")
    s = ii + jj
    inside = (ii >= 1) & (ii <= nx) & (jj >= 1) & (jj <= ny)
    inside[0, :] = inside[-1, :] = False
    owned = inside & (jj >= j0) & (jj <= j1)
    ee, ew, en = (ii < nx).astype(float), (ii > 1).astype(float), (jj < ny).astype(float)
    p = np.zeros_like(f)
    exceed = np.zeros(K + 1, dtype=bool)
    hlast = nx + ny + 2 * (K - 1) + 1  # (the last cell's residual is evaluated one half-sweep after its update)
    for H0 in range(2, hlast + 1, 2 * LEX_NS):
        exchange(p)
        for hh in range(H0, H0 + 2 * LEX_NS):
            before = p.copy()
            pE, pW = np.roll(before, -1, 1), np.roll(before, 1, 1)
            pN, pS = np.roll(before, -1, 0), np.roll(before, 1, 0)
            upd = inside & ((s & 1) == (hh & 1)) & (s <= hh) & (hh <= s + 2 * (K - 1))
            p = np.where(upd, _lex_formula(before, pE, pW, pN, pS, f, ee, ew, en, omega, h), before)
            # residuals of the cells updated in half-sweep hh - 1 (iteration k)
            k = (hh - 1 - s) // 2 + 1
            ev = owned & ((s & 1) != (hh & 1)) & (k >= 1) & (k <= K) & (s <= hh - 1)
            r = _lex_res(before, np.roll(p, -1, 1), pW, np.roll(p, -1, 0), pS, f, ee, ew, en, h)
            hit = ev & (np.abs(r) > tol)
            exceed[np.unique(k[hit])] = True
    bits = ormax(exceed[1:].astype(np.float64))  # OR over the ranks
    stop = next((k for k in range(1, K) if not bits[k - 1] > 0.0), K)
    return j0, j1, p[HALO:-HALO].copy(), stop


def _lex_worker(rank, world, port, q, nx, ny, K, tol):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    try:
        def exchange(p):
            if rank > 0:
                dist.send(torch.from_numpy(p[HALO:2 * HALO].copy()), rank - 1)
                buf = torch.empty((HALO, p.shape[1]), dtype=torch.float64); dist.recv(buf, rank - 1)
                p[:HALO] = buf.numpy()
            if rank < world - 1:
                buf = torch.empty((HALO, p.shape[1]), dtype=torch.float64); dist.recv(buf, rank + 1)
                dist.send(torch.from_numpy(p[-2 * HALO:-HALO].copy()), rank + 1)
                p[-HALO:] = buf.numpy()

        def ormax(a):
            t = torch.from_numpy(a.copy())
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return t.numpy()

        f_full = _lex_source(nx, ny)
        h, omega = 1.0 / nx, 1.7
        j0, j1, strip, stop = _lex_skewed(rank, world, nx, ny, f_full, omega, h, K, tol, exchange, ormax)
        if stop < K:  # the stop is replayed: exactly `stop` iterations from the initial field
            j0, j1, strip, _ = _lex_skewed(rank, world, nx, ny, f_full, omega, h, stop, -1.0, exchange, ormax)
        q.put((rank, j0, j1, strip, stop))
    finally:
        dist.destroy_process_group()


def _lex_source(nx, ny):
    rng = np.random.default_rng(11)
    f = np.zeros((ny + 2, nx + 2))
    f[1:ny + 1, 1:nx + 1] = rng.standard_normal((ny, nx))
    return f


@pytest.mark.parametrize("mode", ["capped", "converging"])
def test_two_rank_reference_order_equals_reference_loop(mode):
    """Two gloo ranks of 20 rows, the skewed reference-order launches with the
    halo exchange and the OR-ed exceedance bits (the GPU rank path of
    ordering = lex, ABI 12) against the reference's own loop on one domain:
    the same stop iteration, the same field bit for bit."""
    world, nx, ny, K = 2, 18, 40, 24
    h, omega = 1.0 / nx, 1.7
    f = _lex_source(nx, ny)
    if mode == "capped":
        tol = 0.0
    else:  # a tolerance met first at iteration 15
        res = []
        for k in range(1, K + 1):
            pk, _ = lex_reference(f, nx, ny, omega, h, k, -1.0)
            r = max(abs(_lex_res(pk[j, i], pk[j, i + 1], pk[j, i - 1], pk[j + 1, i], pk[j - 1, i], f[j, i],
                                 float(i < nx), float(i > 1), float(j < ny), h))
                    for j in range(1, ny + 1) for i in range(1, nx + 1))
            res.append(r)
        assert all(a > b for a, b in zip(res, res[1:]))
        tol = 0.5 * (res[13] + res[14])
    ref, kstop = lex_reference(f, nx, ny, omega, h, K, tol)
    if mode == "converging":
        assert kstop == 15
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_lex_worker, args=(r, world, port, q, nx, ny, K, tol)) for r in range(world)]
    for pr in procs:
        pr.start()
    out = sorted(q.get(timeout=300) for _ in range(world))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for rank, j0, j1, strip, stop in out:
        assert stop == kstop
        assert np.array_equal(strip.view(np.int64), ref[j0:j1 + 1].view(np.int64)), rank


# ---- the reference order's sequential sums on ranks (Solver::seq_sum_ranks) ----

def _chain_worker(rank, world, port, q, nx, ny):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    try:
        f = _lex_source(nx, ny)
        j0, j1 = strip_rows(rank, world, ny)
        acc = torch.zeros(1, dtype=torch.float64)
        for r in range(world):  # one round per link, every rank in every round (the loopback transport's rule)
            if r == rank:
                s = float(acc[0]) if rank > 0 else 0.0
                for j in range(j0, j1 + 1):  # the reference's loop order, one rounding per term
                    for i in range(1, nx + 1):
                        s += float(f[j, i])
                acc[0] = s
            if r + 1 < world:
                if rank == r:
                    dist.send(acc, r + 1)
                elif rank == r + 1:
                    dist.recv(acc, r)
        if rank == world - 1:  # the last rank's total back to every rank
            for p in range(world - 1):
                dist.send(acc, p)
        else:
            dist.recv(acc, world - 1)
        q.put((rank, float(acc[0])))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_rank_chained_sequential_sum_equals_one_loop(world):
    """The open cases' source sum (channel-01.cpp:620-628) on ranks in the
    reference's order: rank r continues rank r-1's running sum, the last
    rank's total goes back to all - bit for bit the single loop's sum (a
    per-rank partial sum all-reduced would re-associate it)."""
    nx, ny = 37, 48
    f = _lex_source(nx, ny)
    one = 0.0
    for j in range(1, ny + 1):
        for i in range(1, nx + 1):
            one += float(f[j, i])
    partial = sum(sum(float(f[j, i]) for j in range(a, b + 1) for i in range(1, nx + 1))
                  for a, b in (strip_rows(r, world, ny) for r in range(world)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_chain_worker, args=(r, world, port, q, nx, ny)) for r in range(world)]
    for pr in procs:
        pr.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for _, v in out:
        assert v.hex() == one.hex()
    assert partial != one or world == 1  # (re-associated partial sums differ in the last bits here)
