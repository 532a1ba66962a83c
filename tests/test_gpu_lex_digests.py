"""Steady reference-order launches at the two largest BASELINE sizes, bit for
bit, without the CPU oracle in the loop.

tests/golden/make_lex_digests.py ran the oracle's restatement of the reference
loop (ORC_LEX) once for one capped timestep of the cavity at 4096^2 (K = 4200)
and of the backwards step at 8192x512 (K = 4400) and stored the iteration
count, the residual and sha256 digests of u, v and p. Both caps lie past
(nx+ny)/2, so the GPU step runs the steady poisson_lexw_kernel<*, 4, false, *>
launches (every cell active: the bench's reference_order launches) between
the ramps; the shorter-K tests in test_gpu_lexw.py run ramp launches only.
Reference loops: cavity-01.cpp:635-678, backwards_step-01.cpp:893-939 (with
the solid / ghost refresh :685-740)."""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import cfd_amd as C  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lex_digests.json")


def digest(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<f8").tobytes()).hexdigest()


def _cases():
    return sorted(json.load(open(GOLDEN))) if os.path.exists(GOLDEN) else []


@pytest.mark.parametrize("name", _cases())
def test_steady_lex_step_matches_oracle_digest(name):
    d = json.load(open(GOLDEN))[name]
    kw = dict(d["params"])
    case = kw.pop("case")
    cp = C.make_params(case, **kw)
    g = C.solver_for(cp, ordering="lex", small_solve="off")
    if case == "cavity":
        g.applyBoundaryConditions()
    it, res = g.step()
    tm = g.timing()
    assert C._lib.SOR_KERNEL.get(tm.sor_kernel) == "lexw"
    assert tm.poisson_steady_launches > 0, "the cap must reach the steady launches"
    assert it == d["sor_iterations"]
    assert res.hex() == d["residual"], (res, d["residual_repr"])
    got = {"u": digest(g.field("u")), "v": digest(g.field("v")), "p": digest(g.field("p"))}
    g.close()
    assert got == d["sha256"]


def test_digest_fixture_present():
    assert _cases(), "tests/golden/lex_digests.json missing: run tests/golden/make_lex_digests.py"
