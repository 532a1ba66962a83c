"""Rayleigh-Benard (BASELINE configs[4]) on the GPU against the CPU oracle.

The reference tree has no Rayleigh-Benard solver (only figures), so this case
is PARITY UNPINNED: the oracle (oracle/cfd_oracle.c orc_temperature_bc,
orc_thermal, orc_step case ORC_RBC) is our own restatement of the cavity's
projection step with the lid at rest plus a Boussinesq temperature field, and
the GPU path must reproduce it bit for bit (same red-black SOR order, same
operand order, -ffp-contract=off on both sides). The physics checks
(conduction onset, Nusselt number) are size-independent properties.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import cfd_amd as C  # noqa: E402
import oracle as O  # noqa: E402
from test_gpu_parity import assert_bits, ofield  # noqa: E402
from test_gpu_ranks import run_ranks  # noqa: E402


def rb(**kw):
    kw.setdefault("nx", 96)
    kw.setdefault("ny", 24)
    kw.setdefault("ra", 2e4)
    kw.setdefault("max_iters", 600)
    return C.make_params("rayleigh_benard", **kw)


def test_initial_temperature_matches_oracle():
    cp = rb()
    g = C.RayleighBenardSolver(cp, ordering="rb")
    o = O.Oracle(cp, ordering=O.RB)
    assert_bits(g.field("t"), o.field("t"), "T0")


def test_stages_bit_exact():
    """One step stage by stage: velocity BCs, predictor, thermal, source, SOR, correction."""
    cp = rb()
    g = C.RayleighBenardSolver(cp, ordering="rb")
    o = O.Oracle(cp, ordering=O.RB)
    g.applyBoundaryConditions()
    o.velocity_bc()
    g.computeTentativeVelocities()
    o.tentative()
    g.advanceTemperature()
    o.temperature_bc()
    o.thermal()
    assert_bits(g.field("vs"), ofield(o, "vs", cp), "v* with buoyancy")
    T = g.field("t")
    assert_bits(T[1:-1, 1:-1], o.field("t")[1:-1, 1:-1], "T after one update")
    g.buildSourceTerm()
    o.source()
    assert_bits(g.field("src")[1:-1, 1:-1], o.field("src")[1:-1, 1:-1], "source")
    gi, gr = g.solverPressurePoisson()
    oi, orr = o.poisson()
    assert (gi, gr) == (oi, orr)
    g.applyPressureCorrection()
    o.correct()
    for f in ("u", "v", "p"):
        assert_bits(g.field(f), ofield(o, f, cp), f)


@pytest.mark.parametrize("n_strips", [1, 3])
def test_steps_bit_exact(n_strips):
    cp = rb(nx=64, ny=48)
    g = C.RayleighBenardSolver(cp, ordering="rb", n_strips=n_strips)
    o = O.Oracle(cp, ordering=O.RB)
    for k in range(12):
        gs = g.step()
        os_ = o.step()
        assert gs == os_, (k, gs, os_)
    for f in ("u", "v", "p"):
        assert_bits(g.field(f), ofield(o, f, cp), f)
    assert_bits(g.field("t")[1:-1, 1:-1], o.field("t")[1:-1, 1:-1], "T")
    assert g.nusselt() == pytest.approx(o.nusselt(), rel=1e-13)  # numpy mean vs sequential sum
    md, ke = g.statistics()
    omd, oke = o.stats()
    assert md == omd and ke == pytest.approx(oke, rel=1e-12)


def test_rank_path_equals_single_domain():
    """Loopback ranks (the RCCL code path) == one domain, bit for bit."""
    cp = rb(nx=64, ny=64)
    res = run_ranks(cp, 2, 8)
    s = C.RayleighBenardSolver(cp, ordering="rb")
    its = [s.step() for _ in range(8)]
    assert res[0]["its"] == its and res[1]["its"] == its
    p = s.field("p")
    for r in res:
        a, b = r["rows"]
        lo = 0 if a == 1 else a
        hi = b + 1 if b == cp.ny else b
        assert_bits(r["p"], p[lo: hi + 1], f"rank rows {a}-{b} p")


def test_onset_and_heat_transport():
    """Above Ra_c the conduction state grows into rolls (kinetic energy rises,
    Nu > 1); below it the perturbation decays (Nu -> 1)."""
    out = {}
    for ra in (1e3, 5e4):
        cp = rb(nx=64, ny=16, ra=ra, max_iters=2000)
        g = C.RayleighBenardSolver(cp, ordering="rb")
        ke = []
        for n in range(1200):
            g.step()
            if n in (200, 1199):
                ke.append(g.statistics()[1])
        out[ra] = (ke, g.nusselt())
    (ke_lo, nu_lo), (ke_hi, nu_hi) = out[1e3], out[5e4]
    assert ke_lo[1] < ke_lo[0] and abs(nu_lo - 1.0) < 1e-2, out
    assert ke_hi[1] > 10 * ke_hi[0] and nu_hi > 1.05, out
