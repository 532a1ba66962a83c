"""Host-side mirror of the reference solver classes over libcfd_amd.so.

CavitySolver / ChannelSolver / BackwardsStepSolver expose the reference's
method names (cavity-01.cpp:306-775, channel-01.cpp:284-770,
backwards_step-01.cpp:316-1062); every method is one or a few C-ABI calls
that launch HIP kernels on the solver's stream. Fields come back as numpy
arrays in the reference's array shapes.
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

from . import _lib
from .logfmt import step_line, warning_line
from .params import BACKSTEP, CASE_NAMES, CAVITY, CHANNEL, RAYLEIGH_BENARD, CaseParams, make_params


def to_cparams(cp: CaseParams, check_every: int = 1, chunk: int = 0, ordering: str = "lex",
               sweeps_per_launch: int = 0, proof_test: str = "auto", small_solve: str = "auto",
               overlap: str = "auto") -> _lib.CfdParams:
    """Derived reference constants -> the C-ABI parameter block. proof_test /
    small_solve / overlap: "auto", "on" or "off" (enum cfd_switch; they choose
    how a solve runs, never its result bits)."""
    return _lib.CfdParams(
        cp.case_id, cp.nx, cp.ny, cp.length, cp.height, cp.re, cp.u_ref, cp.rho, cp.cfl, cp.final_time,
        cp.dx, cp.dy, cp.nu, cp.dt, cp.omega, cp.tol_factor, cp.abs_tol, cp.max_iters, cp.total_steps,
        cp.print_interval, cp.save_interval, cp.h_inlet, cp.step_x, cp.step_i, cp.inlet_jmax, check_every, chunk,
        _lib.ORDER[ordering], sweeps_per_launch, cp.ra, cp.pr, cp.kappa, cp.buoyancy, cp.t_hot, cp.t_cold,
        cp.t_ref, cp.t_perturb, _lib.SWITCH[proof_test], _lib.SWITCH[small_solve], _lib.SWITCH[overlap])


class _SolverBase:
    CASE = CAVITY
    VTK_BASE = "cavity_flow"
    COLLECTION = "cavity_flow_animation.pvd"

    def __init__(self, params: CaseParams | None = None, *, device: int = 0, n_strips: int = 1,
                 check_every: int = 1, chunk: int = 0, rank_rows: tuple[int, int] | None = None, comm=None,
                 ordering: str = "auto", sweeps_per_launch: int = 0, proof_test: str = "auto",
                 small_solve: str = "auto", overlap: str = "auto", tuning: dict[str, int] | None = None):
        """ordering: "lex" (the reference's lexicographic sweep, bit-identical to the
        reference binaries on one device, on strips and on ranks), "rb" (red-black SOR)
        or "auto" (lex; Rayleigh-Benard, which has no reference solver: rb).
        sweeps_per_launch: SOR iterations fused per kernel launch (0 = auto: red-black
        4 in proof-mode launches (the step on strips or ranks: 3), 3 (cavity) / 2 (open
        cases) in exact ones; lexicographic 4, 3 on strips); bit-identical either way.
        proof_test / small_solve / overlap: "auto" / "on" / "off" (include/cfd_amd.h).
        tuning: launch-planning knobs (_lib.TUNING names), performance only."""
        self.params = params if params is not None else make_params(self.CASE)
        if self.params.case_id != self.CASE:
            raise ValueError(f"{type(self).__name__} needs case {CASE_NAMES[self.CASE]}")
        if ordering == "auto":
            ordering = "rb" if self.CASE == RAYLEIGH_BENARD else "lex"
        self.ordering = ordering
        self._cp = to_cparams(self.params, check_every, chunk, ordering, sweeps_per_launch, proof_test,
                              small_solve, overlap)
        L = _lib.lib()
        if rank_rows is None:
            self._h = L.cfd_create(ctypes.byref(self._cp), device, n_strips)
        else:
            self._h = L.cfd_create_rank(ctypes.byref(self._cp), device, rank_rows[0], rank_rows[1], comm)
        if not self._h:
            raise _lib.CfdError("cfd_create failed: " + L.cfd_last_error().decode(errors="replace"))
        for knob, value in (tuning or {}).items():
            self.set_tuning(knob, value)

    def set_tuning(self, knob: str, value: int) -> None:
        """cfd_set_tuning: a launch-planning knob (performance only, same bits)."""
        _lib.check(_lib.lib().cfd_set_tuning(self._h, _lib.TUNING[knob], int(value)), "cfd_set_tuning")

    def close(self) -> None:
        if getattr(self, "_h", None):
            _lib.lib().cfd_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- reference methods -------------------------------------------------
    def applyBoundaryConditions(self) -> None:
        _lib.check(_lib.lib().cfd_apply_bc(self._h), "applyBoundaryConditions")

    def applyTentativeBoundaryConditions(self) -> None:
        _lib.check(_lib.lib().cfd_apply_tentative_bc(self._h), "applyVelocityBC(u*, v*)")

    def computeTentativeVelocities(self) -> None:
        _lib.check(_lib.lib().cfd_compute_tentative(self._h), "computeTentativeVelocities")

    def buildSourceTerm(self) -> None:
        _lib.check(_lib.lib().cfd_build_source(self._h), "buildSourceTerm")

    def solverPressurePoisson(self) -> tuple[int, float]:
        info = _lib.StepInfo()
        _lib.check(_lib.lib().cfd_solve_pressure(self._h, ctypes.byref(info)), "solverPressurePoisson")
        return info.sor_iterations, info.residual

    def applyPressureCorrection(self) -> None:
        _lib.check(_lib.lib().cfd_apply_correction(self._h), "applyPressureCorrection")

    def step(self) -> tuple[int, float]:
        info = _lib.StepInfo()
        _lib.check(_lib.lib().cfd_step(self._h, ctypes.byref(info)), "step")
        return info.sor_iterations, info.residual

    def run_steps(self, n: int) -> tuple[int, float]:
        info = _lib.StepInfo()
        _lib.check(_lib.lib().cfd_run_steps(self._h, n, ctypes.byref(info)), "run_steps")
        return info.sor_iterations, info.residual

    def statistics(self) -> tuple[float, float]:
        """(max divergence, average kinetic energy) as logStatistics computes them."""
        st = _lib.Stats()
        _lib.check(_lib.lib().cfd_compute_stats(self._h, ctypes.byref(st)), "logStatistics")
        return st.max_divergence, st.avg_kinetic_energy

    def interpolateToCellCenters(self) -> tuple[np.ndarray, np.ndarray]:
        self.statistics()
        return self.field("uc"), self.field("vc")

    # ---- fields --------------------------------------------------------------
    def field_shape(self, name: str) -> tuple[int, int]:
        r, c = ctypes.c_int(), ctypes.c_int()
        _lib.check(_lib.lib().cfd_field_shape(self._h, _lib.CFD_FIELD[name], ctypes.byref(r), ctypes.byref(c)),
                   "cfd_field_shape")
        return r.value, c.value

    def field(self, name: str) -> np.ndarray:
        shape = self.field_shape(name)
        out = np.empty(shape, dtype=np.float64)
        _lib.check(_lib.lib().cfd_get_field(self._h, _lib.CFD_FIELD[name],
                                            out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), out.size),
                   "cfd_get_field")
        return out

    def set_field(self, name: str, value: np.ndarray) -> None:
        shape = self.field_shape(name)
        a = np.ascontiguousarray(value, dtype=np.float64)
        if a.shape != shape:
            raise ValueError(f"field {name} expects shape {shape}, got {a.shape}")
        _lib.check(_lib.lib().cfd_set_field(self._h, _lib.CFD_FIELD[name],
                                            a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), a.size),
                   "cfd_set_field")

    def owned_rows(self) -> tuple[int, int]:
        a, b = ctypes.c_int(), ctypes.c_int()
        _lib.check(_lib.lib().cfd_owned_rows(self._h, ctypes.byref(a), ctypes.byref(b)), "cfd_owned_rows")
        return a.value, b.value

    def timing(self) -> _lib.Timing:
        t = _lib.Timing()
        _lib.check(_lib.lib().cfd_get_timing(self._h, ctypes.byref(t)), "cfd_get_timing")
        return t

    def reset_timing(self) -> None:
        _lib.check(_lib.lib().cfd_reset_timing(self._h), "cfd_reset_timing")

    def synchronize(self) -> None:
        _lib.check(_lib.lib().cfd_synchronize(self._h), "cfd_synchronize")

    # ---- output ----------------------------------------------------------------
    def write_vtk(self, filename: str, time_value: float) -> None:
        _lib.check(_lib.lib().cfd_write_vtk(self._h, filename.encode(), time_value), "write_structured_grid")

    def run(self, output_directory: str | None = "vtk_output", out=sys.stdout, err=sys.stderr,
            steps: int | None = None) -> None:
        """The reference's run() (cavity-01.cpp:374-411, channel-01.cpp:360-396)."""
        p = self.params
        total = p.total_steps if steps is None else steps
        files, times = [], []

        def export(k: int, t: float) -> None:
            if output_directory is None:
                return
            name = f"{self.VTK_BASE}_{k:06d}.vtk"
            self.write_vtk(os.path.join(output_directory, name), t)
            files.append(name)
            times.append(t)

        if output_directory is not None:
            os.makedirs(output_directory, exist_ok=True)
        if self.CASE in (CAVITY, RAYLEIGH_BENARD):
            self.applyBoundaryConditions()
        export(0, 0.0)
        for k in range(1, total + 1):
            t = k * p.dt
            it, res = self.step()
            if it >= p.max_iters:
                print(warning_line(p.case_id, p.max_iters, res), file=err)
            if k % p.print_interval == 0 or k == total:
                md, ke = self.statistics()
                nu = self.nusselt() if p.case_id == RAYLEIGH_BENARD else None
                print(step_line(p.case_id, k, p.total_steps, t, md, ke, it, res, nu), file=out)
            if k % p.save_interval == 0 or k == total:
                export(k, t)
        if output_directory is not None:
            write_pvd(os.path.join(output_directory, self.COLLECTION), files, times)


class CavitySolver(_SolverBase):
    CASE = CAVITY
    VTK_BASE = "cavity_flow"
    COLLECTION = "cavity_flow_animation.pvd"


class ChannelSolver(_SolverBase):
    CASE = CHANNEL
    VTK_BASE = "channel_flow"
    COLLECTION = "channel_flow_animation.pvd"


class BackwardsStepSolver(_SolverBase):
    CASE = BACKSTEP
    VTK_BASE = "backwards_step"
    COLLECTION = "backwards_step_animation.pvd"


class RayleighBenardSolver(_SolverBase):
    """BASELINE configs[4] (no reference solver): the cavity's projection step
    with the lid at rest plus a Boussinesq temperature field."""
    CASE = RAYLEIGH_BENARD
    VTK_BASE = "rayleigh_benard"
    COLLECTION = "rayleigh_benard_animation.pvd"

    def advanceTemperature(self) -> None:
        _lib.check(_lib.lib().cfd_advance_temperature(self._h), "advanceTemperature")

    def nusselt(self) -> float:
        """Mean wall-normal conductive flux at the hot wall over dT/H (one-sided)."""
        T = self.field("t")
        p = self.params
        if self.owned_rows()[0] != 1:
            raise ValueError("nusselt() needs the bottom wall (rank owning row 1)")
        return float(np.mean((p.t_hot - T[1, 1:-1]) / (0.5 * p.dy)) / (p.t_hot - p.t_cold))


SOLVERS = {CAVITY: CavitySolver, CHANNEL: ChannelSolver, BACKSTEP: BackwardsStepSolver,
           RAYLEIGH_BENARD: RayleighBenardSolver}


def solver_for(params: CaseParams, **kw) -> _SolverBase:
    return SOLVERS[params.case_id](params, **kw)


def write_pvd(filename: str, files: list[str], times: list[float]) -> None:
    arr = (ctypes.c_char_p * len(files))(*[f.encode() for f in files])
    t = (ctypes.c_double * len(times))(*times)
    _lib.check(_lib.lib().cfd_write_pvd(filename.encode(), arr, t, len(files)), "write_paraview_collection")


def write_vtk_arrays(params: CaseParams, filename: str, time_value: float, uc: np.ndarray, vc: np.ndarray,
                     p: np.ndarray) -> None:
    """Host-only VTK formatting (no device needed): arrays are (ny+2, nx+2)."""
    cp = to_cparams(params)
    shape = (params.ny + 2, params.nx + 2)
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (uc, vc, p)]
    for a in arrs:
        if a.shape != shape:
            raise ValueError(f"expected {shape}, got {a.shape}")
    ptrs = [a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)) for a in arrs]
    _lib.check(_lib.lib().cfd_write_vtk_arrays(ctypes.byref(cp), filename.encode(), time_value, *ptrs),
               "write_structured_grid")


def params_from_library_rb(ra: float, pr: float, nx: int = 0, ny: int = 0, dt: float = 0.0) -> _lib.CfdParams:
    """The C++ Rayleigh-Benard derivation (cfd_params_init_rb)."""
    out = _lib.CfdParams()
    _lib.check(_lib.lib().cfd_params_init_rb(ra, pr, nx, ny, dt, ctypes.byref(out)), "cfd_params_init_rb")
    return out


def params_from_library(case: int, re: float = 0.0, nx: int = 0, ny: int = 0, dt: float = 0.0) -> _lib.CfdParams:
    """The C++ derivation (cfd_params_init), for cross-checking params.py."""
    out = _lib.CfdParams()
    _lib.check(_lib.lib().cfd_params_init(case, re, nx, ny, dt, ctypes.byref(out)), "cfd_params_init")
    return out
