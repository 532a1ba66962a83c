"""Code provenance of a profiled SOR kernel: a sha256 over the sources of the
translation unit that compiles it (the same dependency lists as the
Makefile's object rules, plus the Makefile for the flags). A PMC traffic file
(profiles/r*_pmc_*.json, scripts/pmc_traffic.py) records the hash of the tree
it was taken on; bench.py reports its traffic only while the hash still
matches the sources of the library that ran (a stale profile gives
`traffic: null`). Host-only; reads files under computational-fluid-dynamics_amd/
and include/."""
from __future__ import annotations

import glob
import hashlib
import os

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")

# kernel name prefix -> translation unit (Makefile: $(SRC)/<tu>.o)
_TU = {
    "poisson_multi_kernel": "solver",
    "poisson_wave_kernel": "solver",
    "poisson_lexw_kernel": "solver",
    "poisson_tile_kernel": "tile",
    "poisson_open_proof_kernel": "open",
    "poisson_resident_kernel": "resident",
}


def tu_sources(tu: str) -> list[str]:
    """The files the Makefile rebuilds `tu`.o from (absolute paths, sorted)."""
    hdr = os.path.join(ROOT, "include", "cfd_amd.h")
    mk = os.path.join(PKG, "Makefile")
    own = os.path.join(CSRC, f"{tu}.hip")
    if tu == "solver":
        deps = glob.glob(os.path.join(CSRC, "*.hpp"))
    elif tu == "tile":
        deps = [os.path.join(CSRC, n) for n in ("tile.hpp", "device.hpp")]
    elif tu == "open":
        deps = [os.path.join(CSRC, n) for n in ("open.hpp", "march.hpp", "device.hpp")]
    elif tu == "resident":
        deps = [os.path.join(CSRC, n) for n in ("resident.hpp", "device.hpp", "internal.hpp")]
    else:
        raise ValueError(f"unknown translation unit {tu!r}")
    return sorted({own, hdr, mk, *deps})


def kernel_tu(kernel: str) -> str | None:
    for prefix, tu in _TU.items():
        if kernel.startswith(prefix):
            return tu
    return None


def source_hash(kernel: str) -> str | None:
    """sha256 over (relative path, contents) of the kernel's translation-unit
    sources; None for a kernel name this table does not know."""
    tu = kernel_tu(kernel)
    if tu is None:
        return None
    h = hashlib.sha256()
    for f in tu_sources(tu):
        h.update(os.path.relpath(f, ROOT).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()
