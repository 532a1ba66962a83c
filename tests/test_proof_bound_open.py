"""CPU check of the open cases' proof-mode inequality (device.hpp
`proof_ratio_gen`, used by tile.hip and open.hip).

Channel / backwards-step SOR (channel-01.cpp:659-666): p' = (1-w) p +
w (S - f) / d with S = idx2 (pE + pW) + idy2 (pN + pS), d = 2 (idx2 + idy2),
the divide correctly rounded (kernels' div_denom == IEEE division). For a
black cell whose four neighbours the refresh leaves alone, the residual the
reference evaluates after the sweep (channel-01.cpp:672-681: (pE - 2p + pW)
idx2 + (pN - 2p + pS) idy2 - f) is K (p' - p) + rounding, K = d (1 - w) / w.
The kernels call a sweep "going on" when
    |p' - p| |K| (1 - 2^-38) > tol + 2^-43 (d P + F)
with P >= 9^NS (max|p_in| + F / d) (the launch's growth bound). Claim: then
some cell's reference residual exceeds tol. numpy float64 arithmetic is
IEEE, i.e. the kernels' bits (-ffp-contract=off). Grids spaced like BASELINE
configs[2] (channel 4096x512) and [3] (step 8192x512) and the reference's
own runs; omega of those runs; magnitudes over 12 decades; tolerances placed
at the cells' own residuals.
"""
from __future__ import annotations

import numpy as np
import pytest

import cfd_amd as C


def spacings():
    out = []
    for case, nx, ny in (("channel", 4096, 512), ("backwards_step", 8192, 512), ("channel", None, None),
                         ("backwards_step", None, None)):
        kw = {} if nx is None else {"nx": nx, "ny": ny}
        cp = C.make_params(case, **kw)
        out.append((cp.dx, cp.dy, cp.omega))
    return out


SPACINGS = spacings()


def sweep(p, f, omega, dx, dy):
    """One red-black iteration of the interior (2 <= i, j <= n-1, so every
    updated cell keeps four interior neighbours), operand order of
    sor_interior<CHANNEL>; returns the field and the black mask."""
    idx2, idy2 = 1.0 / (dx * dx), 1.0 / (dy * dy)
    denom = 2.0 * (idx2 + idy2)
    a1 = 1.0 - omega
    ny, nx = p.shape[0] - 2, p.shape[1] - 2
    jj, ii = np.meshgrid(np.arange(ny + 2), np.arange(nx + 2), indexing="ij")
    inner = (ii >= 2) & (ii <= nx - 1) & (jj >= 2) & (jj <= ny - 1)
    q = p.copy()
    for colour in (0, 1):
        m = inner & (((ii + jj) & 1) == colour)
        pe, pw = np.roll(q, -1, 1), np.roll(q, 1, 1)
        pn, ps = np.roll(q, -1, 0), np.roll(q, 1, 0)
        s = idx2 * (pe + pw) + idy2 * (pn + ps)
        new = a1 * q + omega * ((s - f) / denom)
        q = np.where(m, new, q)
    return q, inner & (((ii + jj) & 1) == 1)


def reference_residual(q, f, dx, dy):
    idx2, idy2 = 1.0 / (dx * dx), 1.0 / (dy * dy)
    pe, pw = np.roll(q, -1, 1), np.roll(q, 1, 1)
    pn, ps = np.roll(q, -1, 0), np.roll(q, 1, 0)
    return (pe - 2.0 * q + pw) * idx2 + (pn - 2.0 * q + ps) * idy2 - f


@pytest.mark.parametrize("sp", range(len(SPACINGS)))
@pytest.mark.parametrize("ns", [1, 3, 4])
@pytest.mark.parametrize("scale", [1e-6, 1.0, 1e6])
def test_open_proof_ratio_implies_reference_goes_on(sp, ns, scale):
    dx, dy, omega = SPACINGS[sp]
    idx2, idy2 = 1.0 / (dx * dx), 1.0 / (dy * dy)
    d = 2.0 * (idx2 + idy2)
    rng = np.random.default_rng(sp * 100 + ns * 10 + int(np.log10(scale) + 7))
    n = 50
    p = rng.uniform(-scale, scale, (n, n))
    f = rng.uniform(-1.0, 1.0, (n, n)) * scale * d * rng.choice([1e-6, 1e-3, 1.0], (n, n))
    pin, F = float(np.abs(p).max()), float(np.abs(f).max())
    K = d * abs(1.0 - omega) / omega
    P = 9.0**ns * (pin + F * (1.0 / d) * (1.0 + 2.0**-50)) * (1.0 + 2.0**-40)
    margin = 2.0**-43 * (d * P + F)
    q = p.copy()
    proven = 0
    for _ in range(ns):
        prev = q
        q, black = sweep(q, f, omega, dx, dy)
        assert np.abs(q).max() <= P
        dcell = np.abs(q - prev)[black]
        r = np.abs(reference_residual(q, f, dx, dy))[black]
        for tol in np.concatenate([np.quantile(r, [0.0, 0.5, 0.9, 1.0]), np.sort(r)[-30:],
                                   np.nextafter(np.sort(r)[-30:], 0)]):
            thr = (tol + margin) / K * (1.0 + 2.0**-38)
            bad = (dcell > thr) & ~(r > tol)  # a cell over the threshold has its own |r| > tol
            assert not bad.any(), (tol, r[bad][:3])
            proven += int((dcell > thr).sum())
    assert proven > 0  # not vacuous


def test_open_identity_residual_is_K_times_update():
    """Exact-arithmetic identity behind the test: r = K (p' - p) for a black
    cell after its update (checked in extended precision, rationals-free)."""
    dx, dy, omega = SPACINGS[0]
    rng = np.random.default_rng(3)
    p = rng.uniform(-1, 1, (20, 20))
    f = rng.uniform(-1, 1, (20, 20)) * 1e6
    q, black = sweep(p, f, omega, dx, dy)
    d = 2.0 * (1.0 / (dx * dx) + 1.0 / (dy * dy))
    K = d * (1.0 - omega) / omega
    r = reference_residual(np.longdouble(q), np.longdouble(f), np.longdouble(dx), np.longdouble(dy))[black]
    kd = (np.longdouble(K) * (np.longdouble(q) - np.longdouble(p)))[black]
    scale = np.abs(r).max() + np.abs(kd).max()
    assert np.abs(r - kd).max() <= 1e-9 * scale
