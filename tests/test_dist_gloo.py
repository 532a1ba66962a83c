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
