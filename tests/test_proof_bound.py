"""CPU check of the proof-mode convergence test's inequality (kernels.hpp
`proof_ratio`, small.hpp; derivation in DESIGN.md §2).

A black cell with four neighbours proves "the reference goes on" when
    |p' - p| |K| (1 - 2^-38) > tol + 2^-43 (idx2 (P + h^2 |f|)(1 + 2^-40) + |f|),
K = 4 idx2 (1 - w) / w, P >= every |value| in its stencil. The claim: then the
reference's own residual of that cell (cavity-01.cpp:659-677, evaluated in
its operand order) exceeds tol. numpy float64 arithmetic is IEEE, so the
update and the residual below are the kernels' bits (the library is built
with -ffp-contract=off). Random fields over several magnitudes, omega from 1
to the 4096^2 optimum, and tolerances placed right at the cells' residuals
(the adversarial case): no proven cell may have |r| <= tol.
"""
from __future__ import annotations

import numpy as np
import pytest


def black_half_sweep(p, f, omega, h):
    """Red then black half-sweep of the interior (cavity interior update,
    sor_interior / cav_edge_sor operand order); returns the field after red,
    after black, and the black mask of four-neighbour cells."""
    h2 = h * h
    om = omega / 4.0
    a1 = 1.0 - omega
    ny, nx = p.shape[0] - 2, p.shape[1] - 2
    jj, ii = np.meshgrid(np.arange(ny + 2), np.arange(nx + 2), indexing="ij")
    inner = (ii >= 2) & (ii <= nx - 1) & (jj >= 2) & (jj <= ny - 1)
    q = p.copy()
    for colour in (0, 1):
        m = inner & (((ii + jj) & 1) == colour)
        pe, pw = np.roll(q, -1, 1), np.roll(q, 1, 1)
        pn, ps = np.roll(q, -1, 0), np.roll(q, 1, 0)
        new = q * a1 + om * ((pe + pw) + (pn + ps) - f * h2)
        q = np.where(m, new, q)
        if colour == 0:
            after_red = q.copy()
    return after_red, q, inner & (((ii + jj) & 1) == 1)


def reference_residual(q, f, h):
    """cavity-01.cpp:659-677 for interior cells (all indicators 1)."""
    idx2 = 1.0 / (h * h)
    pc = q
    pe, pw = np.roll(q, -1, 1), np.roll(q, 1, 1)
    pn, ps = np.roll(q, -1, 0), np.roll(q, 1, 0)
    return idx2 * ((pe - pc) + (pw - pc) + (pn - pc) + (ps - pc)) - f


# h: the 64^2 test grid's spacing, and the spacings of BASELINE configs[1]
# (1024^2) and of the bench (4096^2), where idx2 = 1.7e7 puts the margin
# 2^-43 (idx2 P + F) in a different range (the grid itself stays 64^2: the
# inequality is per cell)
HS = [1.0 / 64, 1.0 / 1024, 1.0 / 4096]


@pytest.mark.parametrize("h", HS)
@pytest.mark.parametrize("scale", [1e-6, 1.0, 1e3, 1e6])
@pytest.mark.parametrize("omega", [1.0 + 2.0**-20, 1.5, 1.9938888033081086, 1.99847])
def test_proven_cells_exceed_tolerance(scale, omega, h):
    rng = np.random.default_rng(int(scale * 7 + omega * 1000 + 1.0 / h) % 2**31)
    n = 66
    idx2 = 1.0 / (h * h)
    h2 = h * h
    p0 = rng.uniform(-scale, scale, (n, n))
    # sources of the residual's own magnitude: r mixes both terms
    f = rng.uniform(-1.0, 1.0, (n, n)) * scale * idx2 * rng.choice([1e-6, 1e-3, 1.0], (n, n))
    after_red, q, black = black_half_sweep(p0, f, omega, h)
    d = np.abs(q - p0)[black]
    r = np.abs(reference_residual(q, f, h))[black]
    # P: the six stencil values (old and new centre, four new-red neighbours)
    st = [np.abs(p0), np.abs(q), np.abs(np.roll(q, -1, 1)), np.abs(np.roll(q, 1, 1)), np.abs(np.roll(q, -1, 0)),
          np.abs(np.roll(q, 1, 0))]
    P = np.max(np.stack(st), axis=0)[black]
    af = np.abs(f)[black]
    kc = 4.0 * idx2 * abs(1.0 - omega) / omega * (1.0 - 2.0**-38)
    lhs = d * kc
    margin = 2.0**-43 * (idx2 * ((P + h2 * af) * (1.0 + 2.0**-40)) + af)
    proven_any = 0
    for tol in np.concatenate([np.quantile(r, [0.0, 0.1, 0.5, 0.9, 1.0]), r[:200], np.nextafter(r[:200], 0)]):
        proven = lhs > tol + margin
        bad = proven & ~(r > tol)
        assert not bad.any(), (tol, r[bad][:3], lhs[bad][:3])
        proven_any += int(proven.sum())
    assert proven_any > 0  # the test is not vacuous


@pytest.mark.parametrize("ns", [3, 4])
@pytest.mark.parametrize("h,omega", [(1.0 / 1024, 1.9938888033081086), (1.0 / 4096, 1.99847)])
@pytest.mark.parametrize("scale", [1e-3, 1.0, 1e4])
def test_kernel_proof_ratio_at_baseline_spacings(ns, h, omega, scale):
    """kernels.hpp proof_ratio exactly as the multi-launch kernel evaluates it
    (global P = 9^NS (max|p_in| + h^2 F)(1 + 2^-40), threshold by division,
    ratio > 1 = proven) after NS sweeps, at the spacings of configs[1] and of
    the bench: a proven sweep must have a black cell whose reference residual
    exceeds tol, for tolerances placed at every quantile of the residuals."""
    rng = np.random.default_rng(int(1.0 / h) + ns + int(scale * 10))
    n = 66
    idx2 = 1.0 / (h * h)
    h2 = h * h
    p = rng.uniform(-scale, scale, (n, n))
    f = rng.uniform(-1.0, 1.0, (n, n)) * scale * idx2 * rng.choice([1e-4, 1e-2, 1.0], (n, n))
    pin, F = float(np.abs(p).max()), float(np.abs(f).max())
    K = 4.0 * idx2 * abs(1.0 - omega) / omega
    growth = 9.0**ns
    P = growth * (pin + h2 * F) * (1.0 + 2.0**-40)
    margin = 2.0**-43 * (idx2 * P + F)
    q = p.copy()
    proven_sweeps = 0
    for _ in range(ns):
        prev = q
        _, q, black = black_half_sweep(q, f, omega, h)
        dmax_cells = np.abs(q - prev)[black]
        r = np.abs(reference_residual(q, f, h))[black]
        assert np.abs(q).max() <= P
        for tol in np.concatenate([np.quantile(r, [0.0, 0.5, 0.9, 0.99, 1.0]), np.sort(r)[-20:]]):
            thr = (tol + margin) / K * (1.0 + 2.0**-38)
            ratio = dmax_cells.max() / thr
            if ratio > 1.0:
                assert (r > tol).any(), (tol, ratio)
                proven_sweeps += 1
            # and per cell: a cell over the threshold has its own |r| > tol
            bad = (dmax_cells > thr) & ~(r > tol)
            assert not bad.any(), (tol, r[bad][:3])
    assert proven_sweeps > 0  # not vacuous: the global margin still lets sweeps prove


@pytest.mark.parametrize("h", [1.0 / 32, 1.0 / 4096])
def test_global_bound_of_the_launch_kernel(h):
    """The multi-launch kernel bounds P per wave: 9^NS (max|p_in| + h^2 F)
    with F = max|f| must cover every value a launch of NS sweeps produces."""
    rng = np.random.default_rng(5)
    n, omega = 34, 1.99
    p = rng.uniform(-1, 1, (n, n))
    f = rng.uniform(-1, 1, (n, n)) * 1e3
    pin, F = np.abs(p).max(), np.abs(f).max()
    for ns in range(1, 5):
        q = p.copy()
        for _ in range(ns):
            _, q, _ = black_half_sweep(q, f, omega, h)
        assert np.abs(q).max() <= 9.0**ns * (pin + h * h * F)
