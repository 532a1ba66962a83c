"""Proof-mode launches of the open cases on the wave march (csrc/open.hip):
four red-black sweeps per launch for the channel and the backwards step, the
ghost / solid refresh taken in the skew (rules reading the cell's own row or
the row the march reached earlier when the row enters the next sweep's
window, rules reading the later row one step after it), and the proof-mode
convergence test with the open cases' K = 2 (idx2 + idy2)(1 - w)/w.

The launch must be invisible: the same iteration counts, residuals and
fields, bit for bit, as exact residuals in every sweep (pair launches) and as
the red-black oracle; converging solves end with an iteration the proof
leaves open (exact fallback)."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import cfd_amd as C  # noqa: E402
import oracle as O  # noqa: E402
from cfd_amd import _lib  # noqa: E402
from test_gpu_parity import assert_bits  # noqa: E402

SOLVERS = {"channel": C.ChannelSolver, "backwards_step": C.BackwardsStepSolver}
FIELDS = ("p", "u", "v")
MARCH = {"tile_rounds": 0, "resident": 0}  # the wave march (the LDS tiles and the resident launch have their own tests)


def run(case, cp, steps, strips=1, **kw):
    g = SOLVERS[case](cp, ordering="rb", device=0, small_solve="off", n_strips=strips, tuning=MARCH, **kw)
    hist = [g.step() for _ in range(steps)]
    out = {n: g.field(n).copy() for n in FIELDS}
    tm = g.timing()
    g.close()
    return hist, out, tm


@pytest.mark.parametrize("case,nx,ny,cap,tolf,steps", [
    ("channel", 400, 96, 3000, 1e-4, 3), ("channel", 700, 300, 400, None, 2), ("channel", 257, 131, 3000, 1e-3, 2),
    ("backwards_step", 400, 100, 3000, 1e-4, 3), ("backwards_step", 900, 260, 300, None, 2),
    ("backwards_step", 517, 131, 2000, 1e-3, 2),
    # column tiles wholly left of the step's column (step_i = nx/4 >= 3 tiles):
    # their own class in the plan, interior-column bands below the block
    ("backwards_step", 1600, 160, 400, None, 2), ("backwards_step", 1800, 200, 3000, 1e-4, 2),
])
def test_open_proof_equals_exact(case, nx, ny, cap, tolf, steps):
    cp = C.make_params(case, nx=nx, ny=ny, max_iters=cap)
    if tolf is not None:
        cp.tol_factor = tolf
    hp, fp, tp = run(case, cp, steps)
    he, fe, te = run(case, cp, steps, proof_test="off")
    assert _lib.SOR_KERNEL[tp.sor_kernel] == "march"
    assert hp == he
    for n in FIELDS:
        assert_bits(fp[n], fe[n], f"{case} {nx}x{ny} proof {n}")
    assert te.proof_fallbacks == 0
    assert tp.poisson_sweeps > 3 * tp.poisson_launches or tp.proof_fallbacks > 0  # 4-sweep launches ran
    if any(h[0] < cap for h in he):
        assert tp.proof_fallbacks >= 1


@pytest.mark.parametrize("case,nx,ny", [("channel", 333, 150), ("backwards_step", 333, 150),
                                        ("backwards_step", 1600, 160)])
@pytest.mark.parametrize("cap", [37, 40, 41])
def test_open_proof_vs_red_black_oracle(case, nx, ny, cap):
    """One solve from a random source and initial pressure (ghosts included),
    capped inside / at the end of a 4-sweep launch: iteration count, residual
    (the final field's: proof launches report it from the field) and p.
    1600x160: the step's left-of-column tile class (plan nl > 0)."""
    cp = C.make_params(case, nx=nx, ny=ny, max_iters=cap)
    rng = np.random.default_rng(11)
    f = rng.standard_normal((cp.ny + 2, cp.nx + 2))
    p0 = rng.standard_normal((cp.ny + 2, cp.nx + 2))
    g = SOLVERS[case](cp, ordering="rb", device=0, small_solve="off", tuning=MARCH)
    o = O.Oracle(cp, ordering=O.RB)
    g.set_field("src", f)
    o.field("src")[...] = f
    g.set_field("p", p0)
    o.field("p")[...] = p0
    assert g.solverPressurePoisson() == o.poisson()
    assert_bits(g.field("p"), o.field("p"), f"{case} p, cap {cap}")
    g.close()


@pytest.mark.parametrize("case,nx", [("channel", 400), ("backwards_step", 400), ("backwards_step", 1600)])
@pytest.mark.parametrize("strips", [2, 3])
def test_open_proof_on_strips(case, nx, strips):
    """Strips on one device (8-row halos exchanged once per launch: the
    4-sweep pipeline's depth is 8). Step 1600 wide: the left-of-column tile
    class on strips below, across and above the block's lower edge."""
    cp = C.make_params(case, nx=nx, ny=240, max_iters=600)
    h1, f1, _ = run(case, cp, 2)
    h2, f2, t2 = run(case, cp, 2, strips=strips)
    assert h1 == h2
    for n in FIELDS:
        np.testing.assert_allclose(f2[n], f1[n], rtol=0, atol=1e-12 * max(1.0, np.abs(f1[n]).max()))


def test_open_proof_full_size_channel_capped():
    """BASELINE configs[2] (channel 4096x512): a capped step, proof vs exact."""
    cp = C.make_params("channel", nx=4096, ny=512, max_iters=300)
    hp, fp, tp = run("channel", cp, 1)
    he, fe, _ = run("channel", cp, 1, proof_test="off")
    assert hp == he
    assert_bits(fp["p"], fe["p"], "channel 4096x512 p")
    assert tp.proof_fallbacks == 0


def test_open_proof_full_size_step_capped():
    """BASELINE configs[3] (step 8192x512, its left-of-column tile class): a
    capped step, proof vs exact."""
    cp = C.make_params("backwards_step", nx=8192, ny=512, max_iters=300)
    hp, fp, tp = run("backwards_step", cp, 1)
    he, fe, _ = run("backwards_step", cp, 1, proof_test="off")
    assert hp == he
    assert_bits(fp["p"], fe["p"], "step 8192x512 p")
    assert tp.proof_fallbacks == 0


@pytest.mark.parametrize("case,nx,ny,cap", [("channel", 400, 240, 600), ("backwards_step", 400, 240, 600),
                                            ("backwards_step", 1600, 160, 400), ("channel", 4096, 512, 200)])
@pytest.mark.parametrize("strips", [2, 3])
def test_open_proof_equals_exact_on_strips(case, nx, ny, cap, strips):
    """The same strip decomposition with and without the proof test: the
    source and its mean are the same bits, so any difference would come from
    the 4-sweep proof launch (8 halo rows, refresh timing at strip edges).
    Iteration counts and fields bit for bit (the step on strips runs 3-sweep
    proof launches; 1600 wide: its left-of-column tile class)."""
    cp = C.make_params(case, nx=nx, ny=ny, max_iters=cap)
    hp, fp, tp = run(case, cp, 2, strips=strips)
    he, fe, te = run(case, cp, 2, strips=strips, proof_test="off")
    assert hp == he
    for n in FIELDS:
        assert_bits(fp[n], fe[n], f"{case} {nx}x{ny} strips {strips} proof vs exact {n}")
    assert te.proof_fallbacks == 0
    assert tp.poisson_sweeps > 2.5 * tp.poisson_launches  # proof launches (3-4 sweeps) ran


@pytest.mark.parametrize("case,nx,ny,cap", [("channel", 400, 240, 600), ("backwards_step", 1600, 160, 400)])
@pytest.mark.parametrize("world", [2, 3])
def test_open_proof_equals_exact_on_ranks(case, nx, ny, cap, world):
    """Loopback ranks (the rank code path: halo exchange, all-reduced proof
    slots), proof test on vs off: the same iterations and fields bit for bit."""
    from test_gpu_ranks import run_ranks
    cp = C.make_params(case, nx=nx, ny=ny, max_iters=cap)
    rp = run_ranks(cp, world, 2, small_solve="off", tuning=MARCH)
    re_ = run_ranks(cp, world, 2, small_solve="off", tuning=MARCH, proof_test="off")
    for a, b in zip(rp, re_):
        assert a["its"] == b["its"] and a["rows"] == b["rows"]
        for n in FIELDS:
            assert_bits(a[n], b[n], f"{case} rank rows {a['rows']} proof vs exact {n}")
