"""The reference order's sequential source sum (seqsum.hip, binade-chunked)
against the plain chain of adds, bit for bit, on crafted sources.

The reference removes the source mean with one running sum in loop order
(channel-01.cpp:620-628, backwards_step-01.cpp:843-866): every partial sum
rounded before the next term. seqsum.hip evaluates chunks of terms as exact
integer sums where the running sum provably stays in one binade and as the
plain chain elsewhere. These tests set u* / v* so that source_kernel forms
chosen terms (wide magnitudes, sign changes, exact ties at the running sum's
unit, solids, a carried start on strips), call buildSourceTerm, and compare
the mean-removed source with numpy: the same per-cell operations, the sum as a
Python loop of float adds (one IEEE rounding per term, the reference's loop).
Reference-sized whole runs and the BASELINE digests cover the real sources
(test_gpu_parity.py, test_gpu_lex_digests.py, test_gpu_lex_ranks.py)."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import cfd_amd as C  # noqa: E402


def expected_source(g, cp, us, vs):
    """source_kernel + the sequential sum + subtract_mean_kernel, on the host."""
    ny, nx = cp.ny, cp.nx
    with np.errstate(invalid="ignore"):
        du = us[1:ny + 1, 1:nx + 1] - us[1:ny + 1, 0:nx]
    dv = vs[1:ny + 1, 1:nx + 1] - vs[0:ny, 1:nx + 1]
    f = (cp.rho / cp.dt) * (du * (1.0 / cp.dx) + dv * (1.0 / cp.dy))
    J, I = np.meshgrid(np.arange(1, ny + 1), np.arange(1, nx + 1), indexing="ij")
    fluid = (I > cp.step_i) | (J <= cp.inlet_jmax) if cp.case_id == 2 else np.ones_like(f, dtype=bool)
    f = np.where(fluid, f, 0.0)
    s = 0.0
    for v in f[fluid].tolist():  # loop order: j outer, i inner (row-major), solids skipped
        s = s + v
    mean = s / float(fluid.sum())
    return np.where(fluid, f - mean, 0.0), fluid, s


def run(case, nx, ny, us_rows, n_strips=1, vs=None):
    cp = C.make_params(case, nx=nx, ny=ny, dt=2.0 ** -10)
    if case == "channel":
        cp.length = float(nx)  # dx = 1: integer u* differences give terms (rho / dt) * du exactly
    cls = {"channel": C.ChannelSolver, "backwards_step": C.BackwardsStepSolver}[case]
    g = cls(cp, ordering="lex", n_strips=n_strips)
    us = np.zeros(g.field_shape("us"))
    us[1:ny + 1, :] = us_rows
    vsf = np.zeros(g.field_shape("vs")) if vs is None else vs
    g.set_field("us", us)
    g.set_field("vs", vsf)
    g.reset_timing()
    g.buildSourceTerm()
    got = g.field("src")[1:ny + 1, 1:nx + 1]
    t = g.timing()
    want, fluid, total = expected_source(g, cp, g.field("us"), g.field("vs"))
    bad = np.count_nonzero(got[fluid].view(np.int64) != want[fluid].view(np.int64))
    return bad, t, total


def rows_from_terms(d, ny, nx):
    """u* rows whose differences are the given per-cell values (as floats)."""
    d = np.asarray(d, dtype=np.float64).reshape(ny, nx)
    return np.concatenate([np.zeros((ny, 1)), np.cumsum(d, axis=1)], axis=1)


@pytest.mark.parametrize("kind", ["drift", "signs", "ties", "halves"])
def test_chunked_sum_equals_plain_chain(kind):
    rng = np.random.default_rng({"drift": 1, "signs": 2, "ties": 3, "halves": 4}[kind])
    ny, nx = 96, 2048
    n = ny * nx
    if kind == "drift":  # the open cases' shape: a steady mean plus noise
        d = -9.7 + rng.normal(0.0, 0.05, n)
    elif kind == "signs":  # sign changes, magnitudes over ~20 binades: many crossings of zero
        d = rng.choice([-1.0, 1.0], n) * np.exp(rng.normal(0.0, 7.0, n))
    elif kind == "ties":  # terms 1024 k: as the sum passes 2^63, 2^64, ... exact ties at its unit
        d = rng.integers(2 ** 36, 2 ** 38, n).astype(np.float64)
    else:  # terms 1024 (k + 1/2): ties once the sum passes 2^62
        d = rng.integers(2 ** 36, 2 ** 38, n) + 0.5
    bad, t, total = run("channel", nx, ny, rows_from_terms(d, ny, nx))
    assert bad == 0, f"{bad} cells differ (sum {total!r})"
    assert t.seqsum_chunks >= (n + 2047) // 2048  # (chunks of at most 2048 terms)
    if kind in ("drift", "ties"):  # the integer path carries most chunks
        assert t.seqsum_serial_chunks <= t.seqsum_chunks // 4, (t.seqsum_serial_chunks, t.seqsum_chunks)


@pytest.mark.parametrize("n_strips", [1, 3])
def test_chunked_sum_backwards_step_solids_and_strips(n_strips):
    """Solid cells (-0.0 terms) and strips continuing the previous strip's sum."""
    rng = np.random.default_rng(5)
    ny, nx = 64, 1000  # 64000 terms: a partial last chunk
    d = -3.3 + rng.normal(0.0, 0.5, ny * nx)
    bad, t, total = run("backwards_step", nx, ny, rows_from_terms(d, ny, nx), n_strips=n_strips)
    assert bad == 0, f"{bad} cells differ (sum {total!r})"
    assert t.seqsum_chunks >= (ny * nx + 2047) // 2048


def test_chunked_sum_carries_non_finite_terms():
    """An infinite term: the chain's own result (inf, then NaN past -inf)."""
    ny, nx = 16, 512
    d = np.full(ny * nx, 1.25)
    d[3000] = np.inf
    d[5000] = -np.inf
    us = rows_from_terms(d, ny, nx)
    cp = C.make_params("channel", nx=nx, ny=ny, dt=2.0 ** -10)
    g = C.ChannelSolver(cp, ordering="lex")
    u = np.zeros(g.field_shape("us"))
    u[1:ny + 1, :] = us
    g.set_field("us", u)
    g.set_field("vs", np.zeros(g.field_shape("vs")))
    g.buildSourceTerm()
    got = g.field("src")[1:ny + 1, 1:nx + 1]
    want, fluid, total = expected_source(g, cp, g.field("us"), g.field("vs"))
    assert np.isnan(total) or np.isinf(total)
    assert np.array_equal(np.isnan(got), np.isnan(want))
