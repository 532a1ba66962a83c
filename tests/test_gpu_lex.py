"""GPU exact mode (ordering="lex"): the reference's own SOR sweep order,
pipelined as a wavefront on the GPU — bit-identical to the reference.

Checked against the oracle's lexicographic path (itself pinned string-exact to
the reference's logs and VTK frames in test_oracle_golden.py) and directly
against the reference's residual logs: every printed field, SOR iteration
counts and capped-solve warnings included.
"""
from __future__ import annotations

import io
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

import cfd_amd as C  # noqa: E402
from cfd_amd.logfmt import step_line, warning_line  # noqa: E402
import oracle as O  # noqa: E402

LOGS = json.load(open(os.path.join(GOLDEN, "ref_logs.json")))


def bits_equal(a, b):
    return np.array_equal(np.asarray(a).view(np.int64), np.asarray(b).view(np.int64))


@pytest.mark.parametrize("case,steps", [("cavity", 30), ("channel", 30), ("backwards_step", 4)])
def test_lex_run_bitexact_vs_oracle(case, steps):
    cp = C.reference_defaults(case)
    g = C.solver_for(cp, ordering="lex")
    o = O.Oracle(cp, ordering=O.LEX)
    o.velocity_bc(False)  # cavity: the step's first BC is idempotent; open cases: constructor BC
    for k in range(steps):
        ig, rg = g.step()
        io_, ro = o.step()
        assert (ig, rg) == (io_, ro), (k, ig, io_, rg, ro)
    nx = cp.nx
    assert bits_equal(g.field("u"), o.field("u")[:, : nx + 1])
    assert bits_equal(g.field("v"), o.field("v")[: cp.ny + 1, :])
    assert bits_equal(g.field("p"), o.field("p"))
    md, ke = g.statistics()
    omd, oke = o.stats()
    assert (md, ke) == (omd, oke)


@pytest.mark.parametrize("case,nsteps", [("cavity", 200), ("channel", 200), ("backwards_step", 20)])
def test_lex_reproduces_reference_logs(case, nsteps):
    """The GPU run prints the reference binary's own log lines, character for character."""
    cp = C.reference_defaults(case)
    g = C.solver_for(cp, ordering="lex")
    out, err = io.StringIO(), io.StringIO()
    g.run(output_directory=None, out=out, err=err, steps=nsteps)
    lines = [l for l in out.getvalue().splitlines() if l.startswith("Step")]
    ref = LOGS[case]["steps"]
    # run() prints the final step too; the reference's lines are at print_interval
    lines = [l for l in lines if int(l.split()[1].split("/")[0]) % cp.print_interval == 0]
    assert lines == ref[: len(lines)] and len(lines) == nsteps // cp.print_interval
    warns = err.getvalue().splitlines()
    assert warns == LOGS[case]["warnings"][: len(warns)]


def test_lex_vtk_frame_byte_identical(tmp_path):
    """Step 100 of the cavity, written by the GPU solver: the reference's own file bytes."""
    import hashlib
    cp = C.reference_defaults("cavity")
    g = C.CavitySolver(cp, ordering="lex")
    g.applyBoundaryConditions()
    g.run_steps(100)
    fn = tmp_path / "f.vtk"
    g.write_vtk(str(fn), 100 * cp.dt)
    assert hashlib.sha256(fn.read_bytes()).hexdigest() == LOGS["cavity"]["vtk_sha256"]["100"]


def test_narrow_step_lex_rejects_strips():
    """A step block one cell wide keeps the one-workgroup reference-order
    kernel (poisson_lex_kernel): one strip only. (Every other geometry runs
    the multi-block march on strips: tests/test_gpu_lexw.py.)"""
    cp = C.make_params("backwards_step", nx=64, ny=32)
    cp.step_x = 1.5 * cp.dx  # step_i = 1
    assert cp.step_i == 1
    with pytest.raises(C._lib.CfdError if hasattr(C, "_lib") else Exception):
        g = C.BackwardsStepSolver(cp, ordering="lex", n_strips=2)
        g.step()
