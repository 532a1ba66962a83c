// params.cpp — the reference's constants and constructor-derived quantities,
// with the drop-in CLI overrides (--Re/--Nx/--Ny/--dt).
//
// Constants: cavity-01.cpp:309-320, channel-01.cpp:287-300,
// backwards_step-01.cpp:319-334. Derivations: cavity-01.cpp:355-363,
// channel-01.cpp:336-344, backwards_step-01.cpp:377-387; SOR factor:
// cavity-01.cpp:74-78 / channel-01.cpp:76-81 (identical for nx == ny).
// Mirrors cfd_amd/params.py (checked equal in tests/test_host_logic.py).
#include <algorithm>
#include <cmath>
#include <cstring>

#include "internal.hpp"

namespace {

double omega_2d(int nx, int ny) {
  const double pi = 3.14159265358979323846;
  const double rho_j = 0.5 * (std::cos(pi / (nx + 1)) + std::cos(pi / (ny + 1)));
  const double denom = 1.0 + std::sqrt(std::max(1e-14, 1.0 - rho_j * rho_j));
  return 2.0 / denom;
}

}  // namespace

extern "C" int cfd_params_init(int case_id, double re, int nx, int ny, double dt, cfd_params* out) {
  if (!out) {
    cfd::set_last_error("null output");
    return CFD_E_ARG;
  }
  cfd_params p;
  std::memset(&p, 0, sizeof p);
  p.case_id = case_id;
  p.check_every = 1;
  p.chunk = 0;
  // the reference's own sweep order (bit-identical output) on one device; the
  // rank path (cfd_create_rank) needs CFD_ORDER_RB
  p.ordering = CFD_ORDER_LEX;
  p.sweeps_per_launch = 0;
  switch (case_id) {
    case CFD_CAVITY:
      p.nx = p.ny = 63; p.length = 1.0; p.height = 1.0; p.re = 1000.0; p.u_ref = 1.0; p.rho = 1.0;
      p.cfl = 0.5; p.final_time = 20.0; p.tol_factor = 1e-9; p.abs_tol = 0.0; p.max_iters = 10000;
      p.print_interval = 100; p.save_interval = 100;
      break;
    case CFD_CHANNEL:
      p.nx = 93; p.ny = 31; p.length = 3.0; p.height = 1.0; p.re = 100.0; p.u_ref = 1.0; p.rho = 1.0;
      p.cfl = 0.25; p.final_time = 10.0; p.tol_factor = 1e-7; p.abs_tol = 1e-10; p.max_iters = 10000;
      p.print_interval = 100; p.save_interval = 100;
      break;
    case CFD_BACKSTEP:
      p.nx = 256; p.ny = 32; p.length = 8.0; p.height = 2.0; p.re = 100.0; p.u_ref = 1.0; p.rho = 1.0;
      p.cfl = 0.2; p.final_time = 15.0; p.tol_factor = 1e-7; p.abs_tol = 1e-10; p.max_iters = 10000;
      p.print_interval = 10; p.save_interval = 10; p.h_inlet = 1.0; p.step_x = 2.0;
      break;
    case CFD_RAYLEIGH_BENARD:
      return cfd_params_init_rb(re, 0.71, nx, ny, dt, out);
    default:
      cfd::set_last_error("unknown case_id");
      return CFD_E_ARG;
  }
  if (re > 0) p.re = re;
  if (nx > 0) p.nx = nx;
  if (ny > 0) p.ny = ny;
  else if (nx > 0 && case_id == CFD_CAVITY) p.ny = nx;
  if (p.nx < 2 || p.ny < 2) {
    cfd::set_last_error("grid must have at least 2 interior cells per direction");
    return CFD_E_ARG;
  }
  if (case_id == CFD_CAVITY) {
    p.height = p.ny * p.length / p.nx;
    p.nu = p.rho * p.u_ref * p.length / p.re;
    p.dx = p.dy = p.length / p.nx;
    const double h = p.dx;
    p.dt = p.cfl * std::min(0.25 * h * h / p.nu, h / p.u_ref);
  } else {
    p.nu = p.u_ref * (case_id == CFD_CHANNEL ? p.height : p.h_inlet) / p.re;
    p.dx = p.length / p.nx;
    p.dy = p.height / p.ny;
    const double h = std::min(p.dx, p.dy);
    p.dt = p.cfl * std::min(0.25 * h * h / p.nu, h / std::max(1e-12, p.u_ref));
  }
  if (dt > 0) p.dt = dt;
  p.omega = omega_2d(p.nx, p.ny);
  p.total_steps = (int)(p.final_time / p.dt);
  if (case_id == CFD_BACKSTEP) {
    p.step_i = (int)(p.step_x / p.dx);
    p.inlet_jmax = (int)(p.h_inlet / p.dy);
    if (p.step_i <= 0 || p.step_i >= p.nx) {
      cfd::set_last_error("Step location is outside computational domain!");
      return CFD_E_ARG;
    }
  } else {
    p.inlet_jmax = p.ny;
  }
  if (!(p.dt > 0)) {
    cfd::set_last_error("Computed time step is non-positive. Check physical parameters!");
    return CFD_E_ARG;
  }
  *out = p;
  return CFD_OK;
}

// Rayleigh-Benard (BASELINE configs[4]; no reference solver, mirrors
// cfd_amd/params.py): free-fall units, H = 1, L = nx/ny, lid at rest.
extern "C" int cfd_params_init_rb(double ra, double pr, int nx, int ny, double dt, cfd_params* out) {
  if (!out) {
    cfd::set_last_error("null output");
    return CFD_E_ARG;
  }
  cfd_params p;
  std::memset(&p, 0, sizeof p);
  p.case_id = CFD_RAYLEIGH_BENARD;
  p.check_every = 1;
  p.ordering = CFD_ORDER_RB;  // (no reference solver to reproduce; BASELINE configs[4] runs on ranks)
  p.nx = nx > 0 ? nx : 256;
  p.ny = ny > 0 ? ny : 64;
  p.ra = ra > 0 ? ra : 1e6;
  p.pr = pr > 0 ? pr : 0.71;
  if (p.nx < 2 || p.ny < 2) {
    cfd::set_last_error("grid must have at least 2 interior cells per direction");
    return CFD_E_ARG;
  }
  p.height = 1.0;
  p.length = p.nx * p.height / p.ny;
  p.re = std::sqrt(p.ra / p.pr);
  p.u_ref = 0.0;
  p.rho = 1.0;
  p.cfl = 0.5;
  p.final_time = 100.0;
  p.tol_factor = 1e-9;
  p.abs_tol = 0.0;
  p.max_iters = 10000;
  p.print_interval = 100;
  p.save_interval = 100;
  p.nu = std::sqrt(p.pr / p.ra);
  p.kappa = 1.0 / std::sqrt(p.ra * p.pr);
  p.buoyancy = 1.0;
  p.t_hot = 1.0;
  p.t_cold = 0.0;
  p.t_ref = 0.5 * (p.t_hot + p.t_cold);
  p.t_perturb = 0.01;
  p.dx = p.dy = p.length / p.nx;
  const double h = p.dx;
  p.dt = dt > 0 ? dt : p.cfl * std::min(0.25 * h * h / std::max(p.nu, p.kappa), h / 1.0);
  p.omega = omega_2d(p.nx, p.ny);
  p.total_steps = (int)(p.final_time / p.dt);
  p.inlet_jmax = p.ny;
  *out = p;
  return CFD_OK;
}

// Launch-plan defaults that do not depend on the device (include/cfd_amd.h
// cfd_tuning_default); Solver::init starts from these. Measured on MI355X
// (DESIGN.md §4): cavity boundary-column bands 80 % of the interior march (open
// cases 45 %); a 16-row band floor for the channel and for every reference-order
// (lexw) march, 24 for the red-black step and cavity marches; reference-order
// wall-tile bands 75 % of the interior band up to 2048 rows, 100 % above
// (channel 160 -> 169, cavity 1024^2 160 -> 178 GLUPS; 4096^2 best at 100:
// profiles/r4_tune); LDS tiles for the cavity only.
extern "C" int cfd_tuning_default(const cfd_params* p, int knob, int* value) {
  if (!p || !value) {
    cfd::set_last_error("null argument");
    return CFD_E_ARG;
  }
  const bool cav = p->case_id == CFD_CAVITY || p->case_id == CFD_RAYLEIGH_BENARD;
  switch (knob) {
    case CFD_TUNE_LEXW_EDGE_PCT: *value = p->ny <= 2048 ? 75 : 100; return CFD_OK;
    case CFD_TUNE_PAIR_EDGE_PCT: *value = cav ? 80 : 45; return CFD_OK;
    case CFD_TUNE_MARCH_MIN_TH: *value = (p->case_id == CFD_CHANNEL || p->ordering == CFD_ORDER_LEX) ? 16 : 24; return CFD_OK;
    case CFD_TUNE_TENT_TH: *value = 64; return CFD_OK;
    case CFD_TUNE_LEXW_RAMP_PCT:  // (the step: ramp bands at least the steady height, 134 -> 140 GLUPS at
                                  // 8192x512; the cavity 4096^2 loses 6 % with it: profiles/r5/*lex*)
      *value = p->case_id == CFD_BACKSTEP ? 100 : 0;
      return CFD_OK;
    case CFD_TUNE_TILE_ROUNDS: *value = cav ? 1 : 0; return CFD_OK;
    case CFD_TUNE_MARCH_ORDER: *value = 0; return CFD_OK;
    case CFD_TUNE_LEXW_LEFT: *value = 1; return CFD_OK;
    case CFD_TUNE_LEXW_UPDOWN: *value = 1; return CFD_OK;
    case CFD_TUNE_RESIDENT:  // (the channel 4096x512: 4.96 vs lexw 10.3, red-black 5.03 vs march 8.15 us per sweep)
      *value = (cav || p->case_id == CFD_CHANNEL) ? 1 : 0;
      return CFD_OK;
    case CFD_TUNE_PAIR_WPS:
    case CFD_TUNE_WAVE_WPS:
    case CFD_TUNE_LEXW_WAVES:
      cfd::set_last_error("this knob's default is derived from the device's occupancy at cfd_create");
      return CFD_E_STATE;
    default:
      cfd::set_last_error("unknown tuning knob");
      return CFD_E_ARG;
  }
}
