/*
 * oracle/cfd_oracle.c — TEST INFRASTRUCTURE ONLY (see cfd_oracle.h).
 *
 * Plain-C restatement of the reference's per-timestep path. Every function
 * cites the reference lines it follows. Floating-point expressions keep the
 * reference's operand order and are compiled with -ffp-contract=off, so the
 * lexicographic path reproduces the reference bit for bit (pinned against the
 * reference's own VTK frames and residual logs in tests/test_oracle_golden.py).
 *
 * ORC_RB restates the GPU's red-black ordering of the same SOR update (same
 * formulas, same ghost/solid refresh after each sweep, same residual), so the
 * HIP kernel can be checked bit-exactly, iteration count included.
 */
#include "cfd_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

struct orc_state {
  orc_params P;
  int W;                      /* row pitch = nx + 2 */
  double* f[ORC_NFIELDS];
  unsigned char* fluid;       /* backwards step mask, (ny+2) x (nx+2) */
  int fluid_count;
};

#define AT(a, j, i) ((a)[(size_t)(j) * (size_t)W + (size_t)(i)])
/* Rayleigh-Benard runs the cavity's projection (all no-slip walls, lid at rest) */
#define CAVLIKE(s) ((s)->P.case_id == ORC_CAVITY || (s)->P.case_id == ORC_RBC)

double orc_omega_square(int n) {
  /* cavity-01.cpp:74-78 */
  const double pi = 3.14159265358979323846;
  const double rho_j = cos(pi / (n + 1));
  return 2.0 / (1.0 + sqrt(1.0 - rho_j * rho_j));
}

double orc_omega_2d(int nx, int ny) {
  /* channel-01.cpp:76-81, backwards_step-01.cpp:77-82 */
  const double pi = 3.14159265358979323846;
  const double rho_j = 0.5 * (cos(pi / (nx + 1)) + cos(pi / (ny + 1)));
  const double t = 1.0 - rho_j * rho_j;
  const double denom = 1.0 + sqrt(t > 1e-14 ? t : 1e-14);
  return 2.0 / denom;
}

orc_state* orc_create(const orc_params* p) {
  if (!p || p->nx <= 0 || p->ny <= 0) return NULL;
  orc_state* s = (orc_state*)calloc(1, sizeof(orc_state));
  if (!s) return NULL;
  s->P = *p;
  s->W = p->nx + 2;
  const size_t n = (size_t)(p->ny + 2) * (size_t)(p->nx + 2);
  for (int k = 0; k < ORC_NFIELDS; ++k) {
    s->f[k] = (double*)calloc(n, sizeof(double));
    if (!s->f[k]) { orc_destroy(s); return NULL; }
  }
  s->fluid = (unsigned char*)calloc(n, 1);
  if (!s->fluid) { orc_destroy(s); return NULL; }
  /* backwards_step-01.cpp:492-520: interior cells are fluid downstream of the
   * step (i > step_i) and in the inlet channel (j <= inlet_jmax); ghosts solid.
   * Channel and cavity: every interior cell is fluid. */
  const int W = s->W;
  int cnt = 0;
  for (int j = 1; j <= p->ny; ++j)
    for (int i = 1; i <= p->nx; ++i) {
      int fl = 1;
      if (p->case_id == ORC_BACKSTEP) fl = (i > p->step_i) || (j <= p->inlet_jmax);
      AT(s->fluid, j, i) = (unsigned char)fl;
      cnt += fl;
    }
  s->fluid_count = cnt;
  if (p->case_id == ORC_RBC) {
    /* conduction profile between the walls plus one roll's perturbation,
     * cell centres x = (i - 1/2) dx, y = (j - 1/2) dy, H = 1 */
    const double pi = 3.14159265358979323846;
    double* T = s->f[ORC_F_T];
    for (int j = 1; j <= p->ny; ++j)
      for (int i = 1; i <= p->nx; ++i) {
        const double x = (i - 0.5) * p->dx, y = (j - 0.5) * p->dy;
        AT(T, j, i) = p->t_hot + (p->t_cold - p->t_hot) * y + p->t_perturb * sin(pi * y) * cos(pi * x / p->length);
      }
  }
  return s;
}

void orc_destroy(orc_state* s) {
  if (!s) return;
  for (int k = 0; k < ORC_NFIELDS; ++k) free(s->f[k]);
  free(s->fluid);
  free(s);
}

double* orc_field(orc_state* s, int which) {
  return (which >= 0 && which < ORC_NFIELDS) ? s->f[which] : NULL;
}
unsigned char* orc_mask(orc_state* s) { return s->fluid; }
int orc_fluid_count(orc_state* s) { return s->fluid_count; }

/* ---------------------------------------------------------------- BCs -- */

static void bc_cavity(orc_state* s) {
  /* cavity-01.cpp:523-543 */
  const int W = s->W, nx = s->P.nx, ny = s->P.ny;
  double* u = s->f[ORC_F_U];
  double* v = s->f[ORC_F_V];
  for (int i = 0; i <= nx; ++i) AT(u, ny + 1, i) = 2.0 * s->P.u_ref - AT(u, ny, i);
  for (int i = 0; i <= nx; ++i) AT(u, 0, i) = -AT(u, 1, i);
  for (int j = 0; j <= ny; ++j) AT(v, j, nx + 1) = -AT(v, j, nx);
  for (int j = 0; j <= ny; ++j) AT(v, j, 0) = -AT(v, j, 1);
}

static void bc_open(orc_state* s, double* u, double* v) {
  /* channel-01.cpp:513-529; backwards_step-01.cpp:616-683 (inlet split at
   * inlet_jmax and the solid-face zeroing loop only for the step). */
  const int W = s->W, nx = s->P.nx, ny = s->P.ny;
  const int step = s->P.case_id == ORC_BACKSTEP;
  const int jin = step ? s->P.inlet_jmax : ny;
  for (int j = 1; j <= jin; ++j) AT(u, j, 0) = s->P.u_ref;
  for (int j = jin + 1; j <= ny; ++j) AT(u, j, 0) = 0.0;
  for (int j = 0; j <= ny; ++j) AT(v, j, 0) = 0.0;
  for (int j = 1; j <= ny; ++j) AT(u, j, nx) = AT(u, j, nx - 1);
  for (int j = 0; j <= ny; ++j) AT(v, j, nx + 1) = AT(v, j, nx);
  for (int i = 1; i <= nx; ++i) AT(v, 0, i) = 0.0;
  for (int i = 0; i <= nx; ++i) AT(u, 0, i) = -AT(u, 1, i);
  for (int i = 1; i <= nx; ++i) AT(v, ny, i) = 0.0;
  for (int i = 0; i <= nx; ++i) AT(u, ny + 1, i) = -AT(u, ny, i);
  if (!step) return;
  const unsigned char* fl = s->fluid;
  for (int j = 1; j <= ny; ++j)
    for (int i = 1; i <= nx; ++i) {
      if (AT(fl, j, i)) continue;
      if (i < nx && AT(fl, j, i + 1)) AT(u, j, i) = 0.0;
      if (i > 1 && AT(fl, j, i - 1)) AT(u, j, i - 1) = 0.0;
      if (j < ny && AT(fl, j + 1, i)) AT(v, j, i) = 0.0;
      if (j > 1 && AT(fl, j - 1, i)) AT(v, j - 1, i) = 0.0;
    }
}

void orc_velocity_bc(orc_state* s, int tentative) {
  if (CAVLIKE(s)) { bc_cavity(s); return; }
  if (tentative) bc_open(s, s->f[ORC_F_US], s->f[ORC_F_VS]);
  else bc_open(s, s->f[ORC_F_U], s->f[ORC_F_V]);
}

/* ----------------------------------------------------------- predictor -- */

void orc_tentative(orc_state* s) {
  /* cavity-01.cpp:548-603, channel-01.cpp:546-603,
   * backwards_step-01.cpp:745-820 (valid-face test). */
  const int W = s->W, nx = s->P.nx, ny = s->P.ny;
  const int step = s->P.case_id == ORC_BACKSTEP;
  const double idx = 1.0 / s->P.dx, idy = 1.0 / s->P.dy;
  const double idx2 = 1.0 / (s->P.dx * s->P.dx), idy2 = 1.0 / (s->P.dy * s->P.dy);
  const double nu = s->P.nu, dt = s->P.dt;
  const double* u = s->f[ORC_F_U];
  const double* v = s->f[ORC_F_V];
  double* us = s->f[ORC_F_US];
  double* vs = s->f[ORC_F_VS];
  const unsigned char* fl = s->fluid;

  for (int j = 1; j <= ny; ++j)
    for (int i = 1; i <= nx - 1; ++i) {
      if (step && !(AT(fl, j, i) || AT(fl, j, i + 1))) { AT(us, j, i) = 0.0; continue; }
      const double c = AT(u, j, i);
      const double diff = nu * ((AT(u, j, i + 1) - 2.0 * c + AT(u, j, i - 1)) * idx2 +
                                (AT(u, j + 1, i) - 2.0 * c + AT(u, j - 1, i)) * idy2);
      const double ue = 0.5 * (c + AT(u, j, i + 1));
      const double uw = 0.5 * (AT(u, j, i - 1) + c);
      const double cx = (ue * ue - uw * uw) * idx;
      const double vn = 0.5 * (AT(v, j, i) + AT(v, j, i + 1));
      const double vso = 0.5 * (AT(v, j - 1, i) + AT(v, j - 1, i + 1));
      const double un = 0.5 * (AT(u, j + 1, i) + c);
      const double uso = 0.5 * (AT(u, j - 1, i) + c);
      const double cy = (vn * un - vso * uso) * idy;
      AT(us, j, i) = c + dt * (diff - cx - cy);
    }

  for (int j = 1; j <= ny - 1; ++j)
    for (int i = 1; i <= nx; ++i) {
      if (step && !(AT(fl, j, i) || AT(fl, j + 1, i))) { AT(vs, j, i) = 0.0; continue; }
      const double c = AT(v, j, i);
      const double diff = nu * ((AT(v, j, i + 1) - 2.0 * c + AT(v, j, i - 1)) * idx2 +
                                (AT(v, j + 1, i) - 2.0 * c + AT(v, j - 1, i)) * idy2);
      const double vn = 0.5 * (c + AT(v, j + 1, i));
      const double vso = 0.5 * (AT(v, j - 1, i) + c);
      const double cy = (vn * vn - vso * vso) * idy;
      const double ue = 0.5 * (AT(u, j, i) + AT(u, j + 1, i));
      const double uw = 0.5 * (AT(u, j, i - 1) + AT(u, j + 1, i - 1));
      const double ve = 0.5 * (c + AT(v, j, i + 1));
      const double vw = 0.5 * (AT(v, j, i - 1) + c);
      const double cx = (ue * ve - uw * vw) * idx;
      AT(vs, j, i) = c + dt * (diff - cy - cx);
    }
}

/* ----------------------------------------------------------- source ---- */

double orc_source(orc_state* s) {
  const int W = s->W, nx = s->P.nx, ny = s->P.ny;
  const double* us = s->f[ORC_F_US];
  const double* vs = s->f[ORC_F_VS];
  double* f = s->f[ORC_F_SRC];
  double max_source = 0.0;
  if (CAVLIKE(s)) {
    /* cavity-01.cpp:613-630 (inside solverPressurePoisson) */
    const double inv = 1.0 / s->P.dx;
    const double dt_inv = 1.0 / s->P.dt;
    for (int j = 1; j <= ny; ++j)
      for (int i = 1; i <= nx; ++i) {
        AT(f, j, i) = dt_inv * s->P.rho *
                      ((AT(us, j, i) - AT(us, j, i - 1)) * inv + (AT(vs, j, i) - AT(vs, j - 1, i)) * inv);
        max_source = fmax(max_source, fabs(AT(f, j, i)));
      }
    return max_source;
  }
  /* channel-01.cpp:608-629, backwards_step-01.cpp:825-866 */
  const int step = s->P.case_id == ORC_BACKSTEP;
  const unsigned char* fl = s->fluid;
  const double idx = 1.0 / s->P.dx, idy = 1.0 / s->P.dy;
  const double coeff = s->P.rho / s->P.dt;
  for (int j = 1; j <= ny; ++j)
    for (int i = 1; i <= nx; ++i) {
      if (step && !AT(fl, j, i)) { AT(f, j, i) = 0.0; continue; }
      AT(f, j, i) = coeff * ((AT(us, j, i) - AT(us, j, i - 1)) * idx + (AT(vs, j, i) - AT(vs, j - 1, i)) * idy);
      max_source = fmax(max_source, fabs(AT(f, j, i)));
    }
  if (max_source > 0) {
    double mean = 0.0;
    int cnt = 0;
    for (int j = 1; j <= ny; ++j)
      for (int i = 1; i <= nx; ++i)
        if (!step || AT(fl, j, i)) { mean += AT(f, j, i); ++cnt; }
    if (cnt > 0) {
      mean /= (double)cnt;
      for (int j = 1; j <= ny; ++j)
        for (int i = 1; i <= nx; ++i)
          if (!step || AT(fl, j, i)) AT(f, j, i) -= mean;
    }
  }
  return max_source;
}

/* ----------------------------------------------------------- Poisson --- */

/* One SOR update of cell (j,i), cavity form: cavity-01.cpp:643-654. */
static inline double cavity_update(const double* p, const double* f, int W, int j, int i, int nx, int ny,
                                   double omega, double h) {
  const int ew = (i > 1) ? 1 : 0;
  const int ee = (i < nx) ? 1 : 0;
  const int en = (j < ny) ? 1 : 0;
  const int es = 1;
  const int nc = ew + ee + en + es;
  return AT(p, j, i) * (1.0 - omega) +
         (omega / nc) * ((ee * AT(p, j, i + 1) + ew * AT(p, j, i - 1)) +
                         (en * AT(p, j + 1, i) + es * AT(p, j - 1, i)) - AT(f, j, i) * (h * h));
}

/* Anisotropic SOR update, channel-01.cpp:659-666 / backwards_step-01.cpp:902-909. */
static inline double open_update(const double* p, const double* f, int W, int j, int i, double omega,
                                 double idx2, double idy2, double denom) {
  const double pW = AT(p, j, i - 1), pE = AT(p, j, i + 1);
  const double pS = AT(p, j - 1, i), pN = AT(p, j + 1, i);
  const double sum = idx2 * (pE + pW) + idy2 * (pN + pS);
  const double gs = (sum - AT(f, j, i)) / denom;
  return (1.0 - omega) * AT(p, j, i) + omega * gs;
}

/* Ghost / solid refresh: channel-01.cpp:531-541, backwards_step-01.cpp:685-740 */
static void pressure_ghosts(orc_state* s, double* p) {
  const int W = s->W, nx = s->P.nx, ny = s->P.ny;
  for (int j = 1; j <= ny; ++j) AT(p, j, 0) = AT(p, j, 1);
  for (int j = 1; j <= ny; ++j) AT(p, j, nx + 1) = 0.0;
  for (int i = 1; i <= nx; ++i) {
    AT(p, 0, i) = AT(p, 1, i);
    AT(p, ny + 1, i) = AT(p, ny, i);
  }
  if (s->P.case_id != ORC_BACKSTEP) return;
  const unsigned char* fl = s->fluid;
  for (int j = 1; j <= ny; ++j)
    for (int i = 1; i <= nx; ++i) {
      if (AT(fl, j, i)) continue;
      double sum = 0.0;
      int n = 0;
      if (i > 1 && AT(fl, j, i - 1)) { sum += AT(p, j, i - 1); n++; }
      if (i < nx && AT(fl, j, i + 1)) { sum += AT(p, j, i + 1); n++; }
      if (j > 1 && AT(fl, j - 1, i)) { sum += AT(p, j - 1, i); n++; }
      if (j < ny && AT(fl, j + 1, i)) { sum += AT(p, j + 1, i); n++; }
      if (n > 0) AT(p, j, i) = sum / n;
    }
}

static double residual_cavity(orc_state* s) {
  /* cavity-01.cpp:659-677 */
  const int W = s->W, nx = s->P.nx, ny = s->P.ny;
  const double* p = s->f[ORC_F_P];
  const double* f = s->f[ORC_F_SRC];
  double* r = s->f[ORC_F_RES];
  const double ih2 = 1.0 / (s->P.dx * s->P.dx);
  double m = 0.0;
  for (int j = 1; j <= ny; ++j)
    for (int i = 1; i <= nx; ++i) {
      const int ew = (i > 1) ? 1 : 0, ee = (i < nx) ? 1 : 0, en = (j < ny) ? 1 : 0, es = 1;
      const double c = AT(p, j, i);
      AT(r, j, i) = ih2 * (ee * (AT(p, j, i + 1) - c) + ew * (AT(p, j, i - 1) - c) + en * (AT(p, j + 1, i) - c) +
                           es * (AT(p, j - 1, i) - c)) -
                    AT(f, j, i);
      m = fmax(m, fabs(AT(r, j, i)));
    }
  return m;
}

static double residual_open(orc_state* s) {
  /* channel-01.cpp:672-681, backwards_step-01.cpp:916-930 */
  const int W = s->W, nx = s->P.nx, ny = s->P.ny;
  const int step = s->P.case_id == ORC_BACKSTEP;
  const unsigned char* fl = s->fluid;
  const double* p = s->f[ORC_F_P];
  const double* f = s->f[ORC_F_SRC];
  double* r = s->f[ORC_F_RES];
  const double idx2 = 1.0 / (s->P.dx * s->P.dx), idy2 = 1.0 / (s->P.dy * s->P.dy);
  double m = 0.0;
  for (int j = 1; j <= ny; ++j)
    for (int i = 1; i <= nx; ++i) {
      if (step && !AT(fl, j, i)) { AT(r, j, i) = 0.0; continue; }
      const double c = AT(p, j, i);
      const double lap = (AT(p, j, i + 1) - 2.0 * c + AT(p, j, i - 1)) * idx2 +
                         (AT(p, j + 1, i) - 2.0 * c + AT(p, j - 1, i)) * idy2;
      AT(r, j, i) = lap - AT(f, j, i);
      m = fmax(m, fabs(AT(r, j, i)));
    }
  return m;
}

/* One full SOR iteration (sweep [+ ghost refresh]) in the requested ordering;
 * returns the max-norm residual of the resulting state. */
static double sor_iteration(orc_state* s, int ordering) {
  const int W = s->W, nx = s->P.nx, ny = s->P.ny;
  double* p = s->f[ORC_F_P];
  const double* f = s->f[ORC_F_SRC];
  const double omega = s->P.omega;
  if (CAVLIKE(s)) {
    const double h = s->P.dx;
    if (ordering == ORC_LEX) {
      for (int j = 1; j <= ny; ++j)
        for (int i = 1; i <= nx; ++i) AT(p, j, i) = cavity_update(p, f, W, j, i, nx, ny, omega, h);
    } else {
      for (int color = 0; color < 2; ++color)
        for (int j = 1; j <= ny; ++j)
          for (int i = 1 + ((j + 1 + color) & 1); i <= nx; i += 2)
            AT(p, j, i) = cavity_update(p, f, W, j, i, nx, ny, omega, h);
    }
    return residual_cavity(s);
  }
  const int step = s->P.case_id == ORC_BACKSTEP;
  const unsigned char* fl = s->fluid;
  const double idx2 = 1.0 / (s->P.dx * s->P.dx), idy2 = 1.0 / (s->P.dy * s->P.dy);
  const double denom = 2.0 * (idx2 + idy2);
  if (ordering == ORC_LEX) {
    for (int j = 1; j <= ny; ++j)
      for (int i = 1; i <= nx; ++i) {
        if (step && !AT(fl, j, i)) continue;
        AT(p, j, i) = open_update(p, f, W, j, i, omega, idx2, idy2, denom);
      }
  } else {
    for (int color = 0; color < 2; ++color)
      for (int j = 1; j <= ny; ++j)
        for (int i = 1 + ((j + 1 + color) & 1); i <= nx; i += 2) {
          if (step && !AT(fl, j, i)) continue;
          AT(p, j, i) = open_update(p, f, W, j, i, omega, idx2, idy2, denom);
        }
  }
  pressure_ghosts(s, p);
  return residual_open(s);
}

static double solve_tolerance(orc_state* s, double* initial) {
  const int W = s->W, nx = s->P.nx, ny = s->P.ny;
  const double* f = s->f[ORC_F_SRC];
  if (CAVLIKE(s)) {
    /* cavity-01.cpp:617-632: tolerance = factor * max|source|, loop primed with 1.0 */
    double m = 0.0;
    for (int j = 1; j <= ny; ++j)
      for (int i = 1; i <= nx; ++i) m = fmax(m, fabs(AT(f, j, i)));
    *initial = 1.0;
    return s->P.tol_factor * m;
  }
  /* channel-01.cpp:642-649, backwards_step-01.cpp:880-890 */
  const int step = s->P.case_id == ORC_BACKSTEP;
  const unsigned char* fl = s->fluid;
  double m = 0.0;
  for (int j = 1; j <= ny; ++j)
    for (int i = 1; i <= nx; ++i)
      if (!step || AT(fl, j, i)) m = fmax(m, fabs(AT(f, j, i)));
  double tol = s->P.tol_factor * (m > 0 ? m : 1.0);
  if (tol < s->P.abs_tol) tol = s->P.abs_tol;
  *initial = tol + 1.0;
  return tol;
}

void orc_poisson(orc_state* s, int ordering, int* iters, double* residual) {
  if (CAVLIKE(s)) {
    /* cavity-01.cpp:610-611: every solve starts from a zero field */
    const size_t n = (size_t)(s->P.ny + 2) * (size_t)(s->P.nx + 2);
    memset(s->f[ORC_F_P], 0, n * sizeof(double));
  }
  double res;
  const double tol = solve_tolerance(s, &res);
  int it = 0;
  /* cavity-01.cpp:635, channel-01.cpp:652, backwards_step-01.cpp:893 */
  while (res > tol && it < s->P.max_iters) {
    ++it;
    res = sor_iteration(s, ordering);
  }
  *iters = it;
  *residual = res;
}

void orc_poisson_fixed(orc_state* s, int ordering, int n_iters, double* residual) {
  double res = 0.0;
  for (int k = 0; k < n_iters; ++k) res = sor_iteration(s, ordering);
  *residual = res;
}

/* ---------------------------------------------------------- corrector -- */

void orc_correct(orc_state* s) {
  const int W = s->W, nx = s->P.nx, ny = s->P.ny;
  const double* p = s->f[ORC_F_P];
  const double* us = s->f[ORC_F_US];
  const double* vs = s->f[ORC_F_VS];
  double* u = s->f[ORC_F_U];
  double* v = s->f[ORC_F_V];
  const double rho = s->P.rho, dt = s->P.dt;
  if (CAVLIKE(s)) {
    /* cavity-01.cpp:695-711 */
    const double dt_over_h = dt / s->P.dx;
    for (int j = 1; j <= ny; ++j)
      for (int i = 1; i <= nx - 1; ++i)
        AT(u, j, i) = AT(us, j, i) - dt_over_h * rho * (AT(p, j, i + 1) - AT(p, j, i));
    for (int j = 1; j <= ny - 1; ++j)
      for (int i = 1; i <= nx; ++i)
        AT(v, j, i) = AT(vs, j, i) - dt_over_h * rho * (AT(p, j + 1, i) - AT(p, j, i));
    return;
  }
  /* channel-01.cpp:693-702, backwards_step-01.cpp:944-976 */
  const int step = s->P.case_id == ORC_BACKSTEP;
  const unsigned char* fl = s->fluid;
  const double cu = dt / (rho * s->P.dx), cv = dt / (rho * s->P.dy);
  for (int j = 1; j <= ny; ++j)
    for (int i = 1; i <= nx - 1; ++i) {
      if (step && !((i == nx - 1) || AT(fl, j, i) || AT(fl, j, i + 1))) { AT(u, j, i) = 0.0; continue; }
      AT(u, j, i) = AT(us, j, i) - cu * (AT(p, j, i + 1) - AT(p, j, i));
    }
  for (int j = 1; j <= ny - 1; ++j)
    for (int i = 1; i <= nx; ++i) {
      if (step && !((j == ny - 1) || AT(fl, j, i) || AT(fl, j + 1, i))) { AT(v, j, i) = 0.0; continue; }
      AT(v, j, i) = AT(vs, j, i) - cv * (AT(p, j + 1, i) - AT(p, j, i));
    }
}

/* ---------------------------------------------------- post-processing -- */

void orc_centers(orc_state* s) {
  /* cavity-01.cpp:717-733, channel-01.cpp:708-724, backwards_step-01.cpp:981-1009 */
  const int W = s->W, nx = s->P.nx, ny = s->P.ny;
  const int step = s->P.case_id == ORC_BACKSTEP;
  const unsigned char* fl = s->fluid;
  const double* u = s->f[ORC_F_U];
  const double* v = s->f[ORC_F_V];
  double* uc = s->f[ORC_F_UC];
  double* vc = s->f[ORC_F_VC];
  if (step) {
    const size_t n = (size_t)(ny + 2) * (size_t)(nx + 2);
    memset(uc, 0, n * sizeof(double));
    memset(vc, 0, n * sizeof(double));
  }
  for (int j = 1; j <= ny; ++j)
    for (int i = 1; i <= nx; ++i)
      if (!step || AT(fl, j, i)) AT(uc, j, i) = 0.5 * (AT(u, j, i - 1) + AT(u, j, i));
  for (int j = 1; j <= ny; ++j)
    for (int i = 1; i <= nx; ++i)
      if (!step || AT(fl, j, i)) AT(vc, j, i) = 0.5 * (AT(v, j - 1, i) + AT(v, j, i));
}

void orc_stats(orc_state* s, double* max_div, double* avg_ke) {
  /* cavity-01.cpp:741-766, channel-01.cpp:733-759, backwards_step-01.cpp:1018-1051 */
  orc_centers(s);
  const int W = s->W, nx = s->P.nx, ny = s->P.ny;
  const int step = s->P.case_id == ORC_BACKSTEP;
  const unsigned char* fl = s->fluid;
  const double* u = s->f[ORC_F_U];
  const double* v = s->f[ORC_F_V];
  const double* uc = s->f[ORC_F_UC];
  const double* vc = s->f[ORC_F_VC];
  double ke = 0.0, md = 0.0;
  int cnt = 0;
  for (int j = 1; j <= ny; ++j)
    for (int i = 1; i <= nx; ++i)
      if (!step || AT(fl, j, i)) {
        ke += 0.5 * (AT(uc, j, i) * AT(uc, j, i) + AT(vc, j, i) * AT(vc, j, i));
        cnt++;
      }
  if (CAVLIKE(s)) {
    const double inv = 1.0 / s->P.dx;
    for (int j = 1; j <= ny; ++j)
      for (int i = 1; i <= nx; ++i) {
        const double d = (AT(u, j, i) - AT(u, j, i - 1) + AT(v, j, i) - AT(v, j - 1, i)) * inv;
        md = fmax(md, fabs(d));
      }
    *avg_ke = ke / (double)(nx * ny);
  } else {
    const double idx = 1.0 / s->P.dx, idy = 1.0 / s->P.dy;
    for (int j = 1; j <= ny; ++j)
      for (int i = 1; i <= nx; ++i)
        if (!step || AT(fl, j, i)) {
          const double d = (AT(u, j, i) - AT(u, j, i - 1)) * idx + (AT(v, j, i) - AT(v, j - 1, i)) * idy;
          md = fmax(md, fabs(d));
        }
    *avg_ke = step ? (cnt > 0 ? ke / cnt : 0.0) : ke / (double)(nx * ny);
  }
  *max_div = md;
}

/* ------------------------------------------------- Rayleigh-Benard ---- */

void orc_temperature_bc(orc_state* s) {
  /* Dirichlet walls by ghost reflection (as the lid, cavity-01.cpp:523-529):
   * hot bottom, cold top; adiabatic sides by ghost copy. Corners unused. */
  const int W = s->W, nx = s->P.nx, ny = s->P.ny;
  double* T = s->f[ORC_F_T];
  for (int i = 1; i <= nx; ++i) {
    AT(T, 0, i) = 2.0 * s->P.t_hot - AT(T, 1, i);
    AT(T, ny + 1, i) = 2.0 * s->P.t_cold - AT(T, ny, i);
  }
  for (int j = 1; j <= ny; ++j) {
    AT(T, j, 0) = AT(T, j, 1);
    AT(T, j, nx + 1) = AT(T, j, nx);
  }
}

void orc_thermal(orc_state* s) {
  /* Boussinesq buoyancy on the v faces, then explicit central advection-
   * diffusion of T with the velocities of the step's start (u_corrected after
   * the wall BCs), conservative face fluxes as in the momentum predictor
   * (cavity-01.cpp:548-603). */
  const int W = s->W, nx = s->P.nx, ny = s->P.ny;
  const double idx = 1.0 / s->P.dx, idy = 1.0 / s->P.dy;
  const double idx2 = 1.0 / (s->P.dx * s->P.dx), idy2 = 1.0 / (s->P.dy * s->P.dy);
  const double dt = s->P.dt, kap = s->P.kappa, b = s->P.buoyancy, tr = s->P.t_ref;
  const double* u = s->f[ORC_F_U];
  const double* v = s->f[ORC_F_V];
  const double* T = s->f[ORC_F_T];
  double* vs = s->f[ORC_F_VS];
  double* T2 = s->f[ORC_F_T2];
  for (int j = 1; j <= ny - 1; ++j)
    for (int i = 1; i <= nx; ++i) AT(vs, j, i) = AT(vs, j, i) + dt * (b * (0.5 * (AT(T, j, i) + AT(T, j + 1, i)) - tr));
  for (int j = 1; j <= ny; ++j)
    for (int i = 1; i <= nx; ++i) {
      const double c = AT(T, j, i);
      const double diff = kap * ((AT(T, j, i + 1) - 2.0 * c + AT(T, j, i - 1)) * idx2 +
                                 (AT(T, j + 1, i) - 2.0 * c + AT(T, j - 1, i)) * idy2);
      const double fe = AT(u, j, i) * (0.5 * (c + AT(T, j, i + 1)));
      const double fw = AT(u, j, i - 1) * (0.5 * (AT(T, j, i - 1) + c));
      const double fn = AT(v, j, i) * (0.5 * (c + AT(T, j + 1, i)));
      const double fs = AT(v, j - 1, i) * (0.5 * (AT(T, j - 1, i) + c));
      AT(T2, j, i) = c + dt * (diff - (fe - fw) * idx - (fn - fs) * idy);
    }
  double* t = s->f[ORC_F_T];
  s->f[ORC_F_T] = s->f[ORC_F_T2];
  s->f[ORC_F_T2] = t;
}

double orc_nusselt(orc_state* s) {
  /* Nu = <-dT/dy>_bottom / ((t_hot - t_cold) / H), one-sided at the wall */
  const int W = s->W, nx = s->P.nx;
  const double* T = s->f[ORC_F_T];
  double q = 0.0;
  for (int i = 1; i <= nx; ++i) q += (s->P.t_hot - AT(T, 1, i)) / (0.5 * s->P.dy);
  return q / nx / (s->P.t_hot - s->P.t_cold);
}

/* ------------------------------------------------------------ timestep -- */

void orc_step(orc_state* s, int ordering, int* iters, double* residual) {
  if (s->P.case_id == ORC_RBC) {
    /* the cavity's order (cavity-01.cpp:387-390) with the thermal stage
     * between predictor and source */
    orc_velocity_bc(s, 0);
    orc_temperature_bc(s);
    orc_tentative(s);
    orc_thermal(s);
    orc_source(s);
    orc_poisson(s, ordering, iters, residual);
    orc_correct(s);
    return;
  }
  if (s->P.case_id == ORC_CAVITY) {
    /* cavity-01.cpp:387-390 */
    orc_velocity_bc(s, 0);
    orc_tentative(s);
    orc_source(s);
    orc_poisson(s, ordering, iters, residual);
    orc_correct(s);
    return;
  }
  /* channel-01.cpp:368-375, backwards_step-01.cpp:412-419 */
  orc_tentative(s);
  orc_velocity_bc(s, 1);
  orc_source(s);
  orc_poisson(s, ordering, iters, residual);
  orc_correct(s);
  orc_velocity_bc(s, 0);
}
