"""Multi-process strip decomposition: host-side plumbing.

One process per GPU. Rank r owns a strip of whole rows of the global grid;
neighbouring strips exchange HALO rows over RCCL inside libcfd_amd.so (the
data path never touches Python). This module only partitions the rows,
bootstraps the RCCL communicator through a torch.distributed group (gloo is
enough: it carries 128 opaque bytes once), and reduces timings.
"""
from __future__ import annotations

import ctypes

HALO = 8  # rows of each neighbour stored per side (csrc/kernels.hpp; a fused SOR pair needs 7)


def strip_rows(rank: int, world: int, ny_global: int) -> tuple[int, int]:
    """Interior rows [first, last] (1-based, inclusive) owned by `rank`: an even
    split of ny_global rows, the remainder spread over the first ranks."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank / world")
    base, extra = divmod(ny_global, world)
    first = 1 + rank * base + min(rank, extra)
    last = first + base - 1 + (1 if rank < extra else 0)
    if last - first + 1 < HALO:
        raise ValueError(f"each rank needs at least {HALO} rows (ny={ny_global}, world={world})")
    return first, last


def weak_rows(rank: int, rows_per_rank: int) -> tuple[int, int]:
    """Weak scaling: every rank owns rows_per_rank rows of a grid of world * rows_per_rank."""
    return rank * rows_per_rank + 1, (rank + 1) * rows_per_rank


def broadcast_comm_id(dist, rank: int, make_id) -> bytes:
    """Rank 0 creates the RCCL unique id (make_id() -> bytes); everyone receives it."""
    obj = [make_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def init_comm(dist, rank: int, world: int, device: int):
    """RCCL communicator for this rank (opaque handle for cfd_create_rank)."""
    from . import _lib

    def make_id() -> bytes:
        buf = (ctypes.c_ubyte * _lib.COMM_ID_BYTES)()
        _lib.check(_lib.lib().cfd_comm_unique_id(buf), "cfd_comm_unique_id")
        return bytes(buf)

    raw = broadcast_comm_id(dist, rank, make_id)
    buf = (ctypes.c_ubyte * _lib.COMM_ID_BYTES).from_buffer_copy(raw)
    comm = _lib.lib().cfd_comm_init(buf, world, rank, device)
    if not comm:
        raise _lib.CfdError("cfd_comm_init: " + _lib.lib().cfd_last_error().decode(errors="replace"))
    return comm


def comm_info(comm) -> dict:
    """What the transport reports about itself (RCCL: ncclCommCount / ncclCommUserRank)."""
    from . import _lib

    n, r, t = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    _lib.check(_lib.lib().cfd_comm_info(comm, ctypes.byref(n), ctypes.byref(r), ctypes.byref(t)), "cfd_comm_info")
    return {"nranks": n.value, "rank": r.value, "transport": "rccl" if t.value == 0 else "loopback"}


def max_over_ranks(dist, value: float) -> float:
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(dist, value: float) -> float:
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
