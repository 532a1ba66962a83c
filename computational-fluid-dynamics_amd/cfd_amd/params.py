"""Case parameters: the reference's hard-coded constants plus the CLI overrides.

The reference solvers take no arguments; their constants live in the solver
classes (cavity-01.cpp:309-320, channel-01.cpp:287-300,
backwards_step-01.cpp:319-334) and the derived quantities are computed in the
constructors (cavity-01.cpp:355-363, channel-01.cpp:336-344,
backwards_step-01.cpp:377-387). This module reproduces both, and lets the
drop-in CLI (--Re/--Nx/--Ny/--dt, README "Run It") override them.

The same derivation is implemented in C++ in csrc/params.cpp for the native
host binaries; tests/test_host_logic.py checks that the two agree.
"""
from __future__ import annotations

import dataclasses
import math

CAVITY, CHANNEL, BACKSTEP, RAYLEIGH_BENARD = 0, 1, 2, 3
CASE_NAMES = {CAVITY: "cavity", CHANNEL: "channel", BACKSTEP: "backwards_step", RAYLEIGH_BENARD: "rayleigh_benard"}
CASE_IDS = {v: k for k, v in CASE_NAMES.items()}


@dataclasses.dataclass
class CaseParams:
    case_id: int
    nx: int
    ny: int
    length: float
    height: float
    re: float
    u_ref: float
    rho: float
    cfl: float
    final_time: float
    tol_factor: float
    abs_tol: float
    max_iters: int
    print_interval: int
    save_interval: int
    # backwards step geometry (case 2)
    h_inlet: float = 0.0
    step_x: float = 0.0
    # overrides (0 = derive as the reference does)
    dt_override: float = 0.0
    omega_override: float = 0.0
    # Rayleigh-Benard (case 3, no reference solver; free-fall units, H = 1)
    ra: float = 0.0
    pr: float = 0.0
    t_hot: float = 1.0
    t_cold: float = 0.0
    t_perturb: float = 0.01

    @property
    def kappa(self) -> float:
        return 1.0 / math.sqrt(self.ra * self.pr) if self.case_id == RAYLEIGH_BENARD else 0.0

    @property
    def buoyancy(self) -> float:
        return 1.0 if self.case_id == RAYLEIGH_BENARD else 0.0

    @property
    def t_ref(self) -> float:
        return 0.5 * (self.t_hot + self.t_cold) if self.case_id == RAYLEIGH_BENARD else 0.0

    # ---- derived, as in the reference constructors ----
    @property
    def nu(self) -> float:
        if self.case_id == RAYLEIGH_BENARD:
            return math.sqrt(self.pr / self.ra)
        if self.case_id == CAVITY:
            return self.rho * self.u_ref * self.length / self.re  # cavity-01.cpp:356
        if self.case_id == CHANNEL:
            return self.u_ref * self.height / self.re  # channel-01.cpp:337
        return self.u_ref * self.h_inlet / self.re  # backwards_step-01.cpp:378

    @property
    def dx(self) -> float:
        return self.length / self.nx

    @property
    def dy(self) -> float:
        if self.case_id in (CAVITY, RAYLEIGH_BENARD):
            return self.length / self.nx  # uniform spacing (cavity-01.cpp:357)
        return self.height / self.ny

    @property
    def omega(self) -> float:
        if self.omega_override > 0:
            return self.omega_override
        return omega_2d(self.nx, self.ny)

    @property
    def dt(self) -> float:
        if self.dt_override > 0:
            return self.dt_override
        nu = self.nu
        if self.case_id == RAYLEIGH_BENARD:  # diffusive and free-fall (U = 1) limits
            h = self.dx
            return self.cfl * min(0.25 * h * h / max(nu, self.kappa), h / 1.0)
        if self.case_id == CAVITY:
            h = self.dx  # cavity-01.cpp:359-360
            return self.cfl * min(0.25 * h * h / nu, h / self.u_ref)
        h = min(self.dx, self.dy)  # channel-01.cpp:341-342
        return self.cfl * min(0.25 * h * h / nu, h / max(1e-12, self.u_ref))

    @property
    def total_steps(self) -> int:
        return int(self.final_time / self.dt)  # cavity-01.cpp:361

    @property
    def step_i(self) -> int:
        return int(self.step_x / self.dx) if self.case_id == BACKSTEP else 0  # backwards_step-01.cpp:386

    @property
    def inlet_jmax(self) -> int:
        return int(self.h_inlet / self.dy) if self.case_id == BACKSTEP else self.ny  # backwards_step-01.cpp:493


def omega_2d(nx: int, ny: int) -> float:
    """channel-01.cpp:76-81; for nx == ny it equals cavity-01.cpp:74-78 exactly."""
    rho_j = 0.5 * (math.cos(math.pi / (nx + 1)) + math.cos(math.pi / (ny + 1)))
    denom = 1.0 + math.sqrt(max(1e-14, 1.0 - rho_j * rho_j))
    return 2.0 / denom


def reference_defaults(case: int | str) -> CaseParams:
    """The reference binaries' hard-coded configuration for each case."""
    if isinstance(case, str):
        case = CASE_IDS[case]
    if case == CAVITY:  # cavity-01.cpp:309-320
        return CaseParams(CAVITY, 63, 63, 1.0, 1.0, 1000.0, 1.0, 1.0, 0.5, 20.0, 1e-9, 0.0, 10000, 100, 100)
    if case == CHANNEL:  # channel-01.cpp:287-300
        return CaseParams(CHANNEL, 93, 31, 3.0, 1.0, 100.0, 1.0, 1.0, 0.25, 10.0, 1e-7, 1e-10, 10000, 100, 100)
    if case == BACKSTEP:  # backwards_step-01.cpp:319-334
        return CaseParams(BACKSTEP, 256, 32, 8.0, 2.0, 100.0, 1.0, 1.0, 0.2, 15.0, 1e-7, 1e-10, 10000, 10, 10,
                          h_inlet=1.0, step_x=2.0)
    if case == RAYLEIGH_BENARD:  # BASELINE configs[4]: Ra 1e6, Pr 0.71, aspect 4 (not in the reference tree)
        return CaseParams(RAYLEIGH_BENARD, 256, 64, 4.0, 1.0, math.sqrt(1e6 / 0.71), 0.0, 1.0, 0.5, 100.0, 1e-9,
                          0.0, 10000, 100, 100, ra=1e6, pr=0.71)
    raise ValueError(f"unknown case {case}")


def make_params(case: int | str, *, re: float | None = None, nx: int | None = None, ny: int | None = None,
                dt: float | None = None, final_time: float | None = None, max_iters: int | None = None,
                omega: float | None = None, ra: float | None = None, pr: float | None = None) -> CaseParams:
    """Reference defaults with the CLI's overrides applied.

    Grid overrides keep the physical domain of the case and change the spacing,
    except the cavity, whose spacing is uniform (h = length / nx) and whose
    height follows ny * h (a square cavity when nx == ny, as in the reference).
    """
    p = reference_defaults(case)
    if re is not None:
        p.re = float(re)
    if nx is not None:
        p.nx = int(nx)
    if ny is not None:
        p.ny = int(ny)
    elif nx is not None and p.case_id == CAVITY:
        p.ny = int(nx)
    if p.case_id == CAVITY:
        p.height = p.ny * p.length / p.nx
    if p.case_id == RAYLEIGH_BENARD:  # H = 1, dx = dy
        p.ra = float(ra if ra is not None else (re if re is not None else p.ra))
        if pr is not None:
            p.pr = float(pr)
        p.re = math.sqrt(p.ra / p.pr)
        p.length = p.nx * p.height / p.ny
    if dt is not None:
        p.dt_override = float(dt)
    if final_time is not None:
        p.final_time = float(final_time)
    if max_iters is not None:
        p.max_iters = int(max_iters)
    if omega is not None:
        p.omega_override = float(omega)
    if p.nx < 2 or p.ny < 2:
        raise ValueError("grid must have at least 2 interior cells per direction")
    if p.case_id == BACKSTEP and not (0 < p.step_i < p.nx):
        raise ValueError("Step location is outside computational domain!")  # backwards_step-01.cpp:459-461
    if p.dt <= 0:
        raise ValueError("Computed time step is non-positive. Check physical parameters!")
    return p
