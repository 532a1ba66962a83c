// march.hpp — the red-black SOR wave-march launches (poisson_wave_kernel,
// poisson_multi_kernel and their device pipelines): templates only, so
// that several translation units may include it (kernels.hpp for the
// solver, open.hip for the open cases' proof-mode launches).
#pragma once

#include "device.hpp"

namespace cfd {

// Every window is a 5-slot ring addressed with compile-time slots and the
// march is unrolled by 5, so rows never move between registers. Slot of the
// row x*d behind the front row R at rotation ROT:
#define CFD_SLOT(X) ((((ROT) + 4 - (X)) % 5 + 10) % 5)

struct WaveRing {
  double2 w[5];   // post-black values, rows R-4d .. R
  double2 q[5];   // final values, rows R-5d .. R-3d
  double2 fr[5];  // source, rows R-d .. R-4d
  double2 np[5];  // prefetched p_in rows R .. R+4d
  double2 nf[5];  // prefetched f rows R-d .. R+3d
  double rmax;
};

template <int CASE>
struct WaveCtx {
  Geo g;
  const Coef& c;  // kernel-argument memory
  const double* pin;
  double* pout;
  __amdgpu_buffer_rsrc_t prs;  // pout as a buffer resource (store_row_pair)
  const double* f;
  int gi, gic, y0, y1, rmin, rmax;
  int py0 = 0, py1 = 0;  // proof mode: rows [py0, py1) whose black cells prove (band rows, 1 <= j < ny)
  // step, interior path over the solid block's lower edge (row-uniform
  // geometry): rows >= uhi are solid (never updated), row blk_row (the first
  // solid row) is refreshed from the fluid row below, residuals up to res_hi
  int uhi = 1 << 30, blk_row = -1, res_hi = 1 << 30;
  // cavity boundary-column waves: the reference's indicator products as lane
  // constants (eps_e, eps_w as 1.0 / 0.0; x * 0.0 == copysign(0, x), the
  // reference's 0 * x, for finite x) and omega / neighbour_count below / at
  // the top row, per column slot (cav_edge_lanes)
  double ce_a = 1.0, cw_a = 1.0, ce_b = 1.0, cw_b = 1.0;
  double om_a = 0.0, om_at = 0.0, om_b = 0.0, om_bt = 0.0;
  bool pair_ok, out_lane, icol_a, icol_b, open_a, open_b;
  __device__ bool fl_a(int j) const { return icol_a && j >= 1 && j <= g.ny && (open_a || j <= c.inlet_jmax); }
  __device__ bool fl_b(int j) const { return icol_b && j >= 1 && j <= g.ny && (open_b || j <= c.inlet_jmax); }
  // boundary-column waves: row and column clamped to stored memory, no select
  // on the value (a select waits for the load and defeats the prefetch): the
  // values of rows / lanes outside the stored grid feed only cells that are
  // never updated, refreshed or stored (ghost rows' refresh reads their inner
  // neighbour; halo lanes' cells are masked)
  __device__ double2 ld(const double* base, int R) const {
    const int Rc = min(max(R, rmin), rmax);
    return *reinterpret_cast<const double2*>(base + (size_t)(Rc - g.row_lo) * (size_t)g.pitch + gic);
  }
  // interior waves: every column stored, rows clamped (wave-uniform scalar math)
  __device__ double2 ld_fast(const double* base, int R) const {
    const int Rc = min(max(R, rmin), rmax);
    const double2* src = reinterpret_cast<const double2*>(base + (size_t)(Rc - g.row_lo) * (size_t)g.pitch + gi);
#if CFD_NT_LOAD  // (A/B build option: streamed loads)
    typedef double d2v __attribute__((ext_vector_type(2)));
    const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(src));
    return make_double2(v.x, v.y);
#else
    return *src;
#endif
  }
};

template <int CASE, int DIR, int ROT>
__device__ __forceinline__ void wave_ring_step(const WaveCtx<CASE>& x, WaveRing& s, int R) {
  const int nx = x.g.nx, ny = x.g.ny;
  const Coef& c = x.c;
  // consume the prefetched row R (and f row R-d); issue the loads 4 rows ahead
  s.w[CFD_SLOT(0)] = s.np[CFD_SLOT(0)];
  s.fr[CFD_SLOT(1)] = s.nf[CFD_SLOT(0)];
  s.np[CFD_SLOT(-4)] = x.ld(x.pin, R + 4 * DIR);
  s.nf[CFD_SLOT(-4)] = x.ld(x.f, R + 3 * DIR);
#define CFD_S(b, a) ((DIR > 0) ? (b) : (a))
#define CFD_N(b, a) ((DIR > 0) ? (a) : (b))
  // red (color 0) at row j = R-d: slot a is red iff j is even
  {
    const int j = R - DIR;
    double2& m = s.w[CFD_SLOT(1)];
    const double2 bh = s.w[CFD_SLOT(2)], ah = s.w[CFD_SLOT(0)];
    const double2 fc = s.fr[CFD_SLOT(1)];
    const double Lb = dpp_from_left(m.y), Ra = dpp_from_right(m.x);
    const bool rowok = j > x.rmin && j < x.rmax;
    if ((j & 1) == 0) {
      const double nv = sor_update<CASE>(c, nx, ny, j, x.gi, m.x, Lb, m.y, CFD_S(bh.x, ah.x), CFD_N(bh.x, ah.x), fc.x);
      m.x = (rowok && x.fl_a(j)) ? nv : m.x;
    } else {
      const double nv =
          sor_update<CASE>(c, nx, ny, j, x.gi + 1, m.y, m.x, Ra, CFD_S(bh.y, ah.y), CFD_N(bh.y, ah.y), fc.y);
      m.y = (rowok && x.fl_b(j)) ? nv : m.y;
    }
  }
  // black (color 1) at row j = R-2d
  {
    const int j = R - 2 * DIR;
    double2& m = s.w[CFD_SLOT(2)];
    const double2 bh = s.w[CFD_SLOT(3)], ah = s.w[CFD_SLOT(1)];
    const double2 fc = s.fr[CFD_SLOT(2)];
    const double Lb = dpp_from_left(m.y), Ra = dpp_from_right(m.x);
    const bool rowok = j > x.rmin && j < x.rmax;
    if ((j & 1) == 1) {
      const double nv = sor_update<CASE>(c, nx, ny, j, x.gi, m.x, Lb, m.y, CFD_S(bh.x, ah.x), CFD_N(bh.x, ah.x), fc.x);
      m.x = (rowok && x.fl_a(j)) ? nv : m.x;
    } else {
      const double nv =
          sor_update<CASE>(c, nx, ny, j, x.gi + 1, m.y, m.x, Ra, CFD_S(bh.y, ah.y), CFD_N(bh.y, ah.y), fc.y);
      m.y = (rowok && x.fl_b(j)) ? nv : m.y;
    }
  }
  // ghost / solid refresh at row j = R-3d (pre-refresh neighbours) -> q
  {
    const double2 m = s.w[CFD_SLOT(3)];
    double2 nv = m;
    if (CASE != CAVITY) {
      const int j = R - 3 * DIR;
      const double2 bh = s.w[CFD_SLOT(4)], ah = s.w[CFD_SLOT(2)];
      const double Lb = dpp_from_left(m.y), Ra = dpp_from_right(m.x);
      double out;
      if (refresh_value<CASE>(c, nx, ny, j, x.gi, m.x, Lb, m.y, CFD_S(bh.x, ah.x), CFD_N(bh.x, ah.x), out)) nv.x = out;
      if (refresh_value<CASE>(c, nx, ny, j, x.gi + 1, m.y, m.x, Ra, CFD_S(bh.y, ah.y), CFD_N(bh.y, ah.y), out))
        nv.y = out;
    }
    s.q[CFD_SLOT(3)] = nv;
  }
  // residual + store at row j = R-4d: q rows R-5d (behind), R-4d, R-3d (ahead)
  {
    const int j = R - 4 * DIR;
    const double2 m = s.q[CFD_SLOT(4)], bh = s.q[CFD_SLOT(5)], ah = s.q[CFD_SLOT(3)];
    const double2 fc = s.fr[CFD_SLOT(4)];
    const double Lb = dpp_from_left(m.y), Ra = dpp_from_right(m.x);
    const bool jout = j >= x.y0 && j < x.y1;
    if (x.out_lane && jout)
      *reinterpret_cast<double2*>(x.pout + (size_t)(j - x.g.row_lo) * (size_t)x.g.pitch + x.gi) = m;
    const bool jres = x.out_lane && jout && j >= x.g.j0 && j <= x.g.j1;
    const double ra = residual_abs<CASE>(c, nx, ny, j, x.gi, m.x, Lb, m.y, CFD_S(bh.x, ah.x), CFD_N(bh.x, ah.x), fc.x);
    const double rb =
        residual_abs<CASE>(c, nx, ny, j, x.gi + 1, m.y, m.x, Ra, CFD_S(bh.y, ah.y), CFD_N(bh.y, ah.y), fc.y);
    s.rmax = fmax(s.rmax, (jres && x.fl_a(j)) ? ra : 0.0);
    s.rmax = fmax(s.rmax, (jres && x.fl_b(j)) ? rb : 0.0);
  }
#undef CFD_S
#undef CFD_N
}

template <int CASE, int DIR>
__device__ __forceinline__ double wave_march_ring(const Geo& g, const Coef& c, const double* __restrict__ pin,
                                                  double* __restrict__ pout, const double* __restrict__ f, int lane,
                                                  int gi, int y0, int y1) {
  constexpr int H = 4;
  WaveCtx<CASE> x{g, c};
  x.pin = pin; x.pout = pout; x.f = f;
  x.prs = out_rsrc(pout, g);
  x.gi = gi;
  x.y0 = y0;
  x.y1 = y1;
  x.rmin = max(g.row_lo, 0);
  x.rmax = min(g.row_lo + g.nrows - 1, g.ny + 1);
  x.pair_ok = gi >= 0 && gi + 1 < g.pitch;
  x.out_lane = x.pair_ok && lane >= H / 2 && lane < 64 - H / 2;
  x.icol_a = gi >= 1 && gi <= g.nx;
  x.icol_b = gi + 1 >= 1 && gi + 1 <= g.nx;
  x.open_a = (CASE != BACKSTEP) || (gi > c.step_i);
  x.open_b = (CASE != BACKSTEP) || (gi + 1 > c.step_i);
  x.gic = min(max(gi, 0), g.pitch - 2);
  const int Rbeg = (DIR > 0) ? y0 - H : y1 - 1 + H;
  const int nsteps = (y1 - y0) + 2 * H;
  WaveRing s;
  const double2 z = make_double2(0.0, 0.0);
#pragma unroll
  for (int k = 0; k < 5; ++k) s.w[k] = s.q[k] = s.fr[k] = z;
  s.rmax = 0.0;
  {
    constexpr int ROT = 0;  // slots as seen by the first step
    s.np[CFD_SLOT(0)] = x.ld(pin, Rbeg);
    s.np[CFD_SLOT(-1)] = x.ld(pin, Rbeg + DIR);
    s.np[CFD_SLOT(-2)] = x.ld(pin, Rbeg + 2 * DIR);
    s.np[CFD_SLOT(-3)] = x.ld(pin, Rbeg + 3 * DIR);
    s.nf[CFD_SLOT(0)] = x.ld(f, Rbeg - DIR);
    s.nf[CFD_SLOT(-1)] = x.ld(f, Rbeg);
    s.nf[CFD_SLOT(-2)] = x.ld(f, Rbeg + DIR);
    s.nf[CFD_SLOT(-3)] = x.ld(f, Rbeg + 2 * DIR);
  }
  int st = 0, R = Rbeg;
  for (; st + 5 <= nsteps; st += 5, R += 5 * DIR) {
    wave_ring_step<CASE, DIR, 0>(x, s, R);
    wave_ring_step<CASE, DIR, 1>(x, s, R + DIR);
    wave_ring_step<CASE, DIR, 2>(x, s, R + 2 * DIR);
    wave_ring_step<CASE, DIR, 3>(x, s, R + 3 * DIR);
    wave_ring_step<CASE, DIR, 4>(x, s, R + 4 * DIR);
  }
  if (st < nsteps) { wave_ring_step<CASE, DIR, 0>(x, s, R); ++st; R += DIR; }
  if (st < nsteps) { wave_ring_step<CASE, DIR, 1>(x, s, R); ++st; R += DIR; }
  if (st < nsteps) { wave_ring_step<CASE, DIR, 2>(x, s, R); ++st; R += DIR; }
  if (st < nsteps) { wave_ring_step<CASE, DIR, 3>(x, s, R); ++st; R += DIR; }
  return s.rmax;
}
#undef CFD_SLOT


template <int CASE>
__global__ __launch_bounds__(256, CFD_WAVE_MIN_WAVES) void poisson_wave_kernel(Geo g, Coef c, const double* __restrict__ pin,
                                                           double* __restrict__ pout, const double* __restrict__ f,
                                                           PoissonCtl ctl, int k, int ka, int kb, int TH, int ctiles,
                                                           int nbands, int flags) {
  constexpr int H = 4, TWC = 128 - 2 * H;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // convergence test of the iterations [ka, kb] (flags bit 2: none - a replay
  // of an iteration already known to be the solve's last)
  if (!(flags & 4) && !window_go_on(ctl, ka, kb, lane, blockIdx.x == 0 && wv == 0, (flags & 128) != 0)) return;

  if (blockIdx.x == 0 && wv == 0 && lane < RES_SHARDS) {  // the next launch's slots (RING_AHEAD)
#pragma unroll
    for (int q = 0; q < RING_AHEAD; ++q)
      ctl.ring[(size_t)((k + 1 + q) & (RING - 1)) * RES_SHARDS * SHARD_STRIDE + lane * SHARD_STRIDE] = 0.0;
  }

  // XCD-aware block order; the 4 waves of a block take 4 adjacent bands
  const int nblk = (int)gridDim.x;
  const int L8 = (nblk / 8) * 8;
  const int bl = (int)blockIdx.x;
  const int blk = ((flags & 2) && bl < L8) ? (bl % 8) * (nblk / 8) + bl / 8 : bl;
  const int tile = blk * 4 + wv;
  if (tile >= ctiles * nbands) return;
  const int band = tile % nbands, ctile = tile / nbands;
  const int gi = ctile * TWC - H + 2 * lane;  // this lane's columns: gi (slot a), gi+1 (slot b)
  const int y0 = g.wj0 + band * TH;
  const int y1 = min(y0 + TH, g.wj1 + 1);
  if (y0 > g.wj1) return;
  double rmaxv = 0.0;
  const bool up = (flags & 1) && (band & 1);
  rmaxv = up ? wave_march_ring<CASE, -1>(g, c, pin, pout, f, lane, gi, y0, y1)
             : wave_march_ring<CASE, 1>(g, c, pin, pout, f, lane, gi, y0, y1);
  rmaxv = wave_max(rmaxv);
  if (lane == 0) {
    double* slot = ctl.ring + (size_t)(k & (RING - 1)) * RES_SHARDS * SHARD_STRIDE;
    atomicMax(reinterpret_cast<unsigned long long*>(slot + (size_t)(tile % RES_SHARDS) * SHARD_STRIDE),
              (unsigned long long)__double_as_longlong(rmaxv));
  }
}

// ------------------------------------- Poisson, two iterations per launch --
//
// Temporal blocking of the wave march: one launch runs SOR iterations k and
// k+1. Iteration k's pipeline is the one above (red at R-1, black at R-2,
// refresh at R-3, residual at R-4; no store); its final rows feed a second
// pipeline, lagging 3 rows (red at R-4, black at R-5, refresh at R-6, residual
// + store at R-7). Every cell sees the same operands in the same order as in
// two single-iteration launches, so the result is bit-identical; the launch
// reads p and f once and writes p once (24 B/cell) for two iterations.
// Dependency depth: 7 rows / columns, so a wave writes 112 of its 128 columns
// (8-column halos) and bands overlap by 7 rows. Both residuals are recorded
// (ring slots k and k+1); if iteration k alone meets the tolerance the host
// replays it with one single-iteration launch from this launch's input.

constexpr int PAIR_H = 7;                     // row / column dependency depth of a pair
constexpr int PAIR_TWC = 128 - 2 * 8;         // output columns per wave (8-column halos)

#define CFD_SLOT(X) ((((ROT) + 4 - (X)) % 5 + 10) % 5)

// NPR: slots of the prefetch rings (rows in flight = NPR - 1); 5 or 10 (the
// unrolled march covers 10 rows, so both return to the same slots)
template <int NPR>
struct WavePair {
  double2 w[5];   // iteration k, post-black rows R-4d .. R
  double2 q[5];   // iteration k, final rows R-5d .. R-3d
  double2 w2[5];  // iteration k+1, post-black rows R-7d .. R-3d
  double2 q2[5];  // iteration k+1, final rows R-8d .. R-6d
  double2 fr[5];  // source rows R-d .. R-5d
  double2 fr2[5]; // source rows R-6d .. R-10d
  double2 np[NPR];  // prefetched p_in rows R .. R+(NPR-1)d
  double2 nf[NPR];  // prefetched f rows R-d .. R+(NPR-2)d
  double rmax1, rmax2;
};

#ifndef CFD_PAIR_NPR
#define CFD_PAIR_NPR 5
#endif


template <int CASE>
struct WaveCtx;

// SOR update of an interior-column cell on an updated row j (row-uniform):
// cavity rows below the top have four neighbours; the top row (j == ny) has
// eps_n = 0 and its north neighbour is the ghost row, which holds +0.0, so the
// reference's 0*p[ny+1][i] equals p[ny+1][i] and only omega/3 differs.
template <int CASE>
__device__ __forceinline__ double sor_fast(const WaveCtx<CASE>& x, int j, double pc, double pW, double pE, double pS,
                                           double pN, double fc) {
  const Coef& c = x.c;
  if (CASE == CAVITY) {
    const double om = (j == x.g.ny) ? c.om_nc[3] : c.om_nc[4];  // row-uniform: a scalar select
    return pc * c.one_m_omega + om * ((pE + pW) + (pN + pS) - fc * c.h2);
  }
  return sor_interior<CASE>(c, pc, pW, pE, pS, pN, fc);
}

// One pipeline stage set of one iteration on ring rows: red at A-d, black at
// A-2d, refresh at A-3d into Q, residual (+ store) at A-4d, where row A-xd of
// W sits in slot CFD_SLOT(x + OFF). FAST: the wave's cells and their
// dependency cone are interior fluid cells of rows that are updated (checked
// per wave by the caller), so no per-cell masks are evaluated; the residual
// of halo lanes is masked once at the end instead of per row.
// RC (FAST only): row checks; without them (bands whose march stays off the
// ghost rows) every row is updated and nothing is refreshed, straight-line
template <int CASE, int DIR, int ROT, int OFF, bool FAST, int APAR, bool RC = true>
__device__ __forceinline__ void pair_stages(const WaveCtx<CASE>& x, double2 (&W)[5], double2 (&Q)[5],
                                            const double2& f_red, const double2& f_black, const double2& f_res,
                                            int A, bool store, double& rm) {
  const int nx = x.g.nx, ny = x.g.ny;
  const Coef& c = x.c;
#define CFD_S(b, a) ((DIR > 0) ? (b) : (a))
#define CFD_N(b, a) ((DIR > 0) ? (a) : (b))
  {  // red (color 0) at row A-d
    const int j = A - DIR;  // parity APAR ^ 1 (compile time)
    double2& m = W[CFD_SLOT(1 + OFF)];
    const double2 bh = W[CFD_SLOT(2 + OFF)], ah = W[CFD_SLOT(0 + OFF)];
    if ((APAR == 2) ? ((j & 1) == 0) : ((APAR ^ 1) == 0)) {  // APAR 2: parity known at run time only
      const double Lb = dpp_from_left(m.y);
      if (FAST) {
        if (!RC || (j > x.rmin && j < x.rmax && j < x.uhi)) m.x = sor_fast<CASE>(x, j, m.x, Lb, m.y, CFD_S(bh.x, ah.x), CFD_N(bh.x, ah.x), f_red.x);
      } else {
        const double nv =
            sor_update<CASE>(c, nx, ny, j, x.gi, m.x, Lb, m.y, CFD_S(bh.x, ah.x), CFD_N(bh.x, ah.x), f_red.x);
        m.x = (j > x.rmin && j < x.rmax && x.fl_a(j)) ? nv : m.x;
      }
    } else {
      const double Ra = dpp_from_right(m.x);
      if (FAST) {
        if (!RC || (j > x.rmin && j < x.rmax && j < x.uhi)) m.y = sor_fast<CASE>(x, j, m.y, m.x, Ra, CFD_S(bh.y, ah.y), CFD_N(bh.y, ah.y), f_red.y);
      } else {
        const double nv =
            sor_update<CASE>(c, nx, ny, j, x.gi + 1, m.y, m.x, Ra, CFD_S(bh.y, ah.y), CFD_N(bh.y, ah.y), f_red.y);
        m.y = (j > x.rmin && j < x.rmax && x.fl_b(j)) ? nv : m.y;
      }
    }
  }
  {  // black (color 1) at row A-2d
    const int j = A - 2 * DIR;  // parity APAR
    double2& m = W[CFD_SLOT(2 + OFF)];
    const double2 bh = W[CFD_SLOT(3 + OFF)], ah = W[CFD_SLOT(1 + OFF)];
    if ((APAR == 2) ? ((j & 1) == 1) : (APAR == 1)) {
      const double Lb = dpp_from_left(m.y);
      if (FAST) {
        if (!RC || (j > x.rmin && j < x.rmax && j < x.uhi)) m.x = sor_fast<CASE>(x, j, m.x, Lb, m.y, CFD_S(bh.x, ah.x), CFD_N(bh.x, ah.x), f_black.x);
      } else {
        const double nv =
            sor_update<CASE>(c, nx, ny, j, x.gi, m.x, Lb, m.y, CFD_S(bh.x, ah.x), CFD_N(bh.x, ah.x), f_black.x);
        m.x = (j > x.rmin && j < x.rmax && x.fl_a(j)) ? nv : m.x;
      }
    } else {
      const double Ra = dpp_from_right(m.x);
      if (FAST) {
        if (!RC || (j > x.rmin && j < x.rmax && j < x.uhi)) m.y = sor_fast<CASE>(x, j, m.y, m.x, Ra, CFD_S(bh.y, ah.y), CFD_N(bh.y, ah.y), f_black.y);
      } else {
        const double nv =
            sor_update<CASE>(c, nx, ny, j, x.gi + 1, m.y, m.x, Ra, CFD_S(bh.y, ah.y), CFD_N(bh.y, ah.y), f_black.y);
        m.y = (j > x.rmin && j < x.rmax && x.fl_b(j)) ? nv : m.y;
      }
    }
  }
  {  // ghost / solid refresh at row A-3d (pre-refresh neighbours) -> Q; none for interior fluid cells
    const double2 m = W[CFD_SLOT(3 + OFF)];
    double2 nv = m;
    if (CASE != CAVITY && FAST && RC) {  // interior columns: only the ghost rows refresh (row-uniform)
      const int j = A - 3 * DIR;
      // values picked at compile time: a ?: between the two ring elements
      // became a select of addresses, which put the whole ring in scratch
      double2 wn, ws;
      if constexpr (DIR > 0) {
        wn = W[CFD_SLOT(2 + OFF)];
        ws = W[CFD_SLOT(4 + OFF)];
      } else {
        wn = W[CFD_SLOT(4 + OFF)];
        ws = W[CFD_SLOT(2 + OFF)];
      }
      if (j == 0) nv = wn;       // p[0][i] = p[1][i]
      if (j == ny + 1) nv = ws;  // p[ny+1][i] = p[ny][i]
      if (CASE == BACKSTEP && j == x.blk_row) {  // backwards_step-01.cpp:708-738: one fluid neighbour (S),
        nv.x = 0.0 + ws.x;                       // the average (0 + p_S) / 1 of the reference
        nv.y = 0.0 + ws.y;
      }
    }
    if (CASE != CAVITY && !FAST) {
      const int j = A - 3 * DIR;
      const double2 bh = W[CFD_SLOT(4 + OFF)], ah = W[CFD_SLOT(2 + OFF)];
      const double Lb = dpp_from_left(m.y), Ra = dpp_from_right(m.x);
      double out;
      if (refresh_value<CASE>(c, nx, ny, j, x.gi, m.x, Lb, m.y, CFD_S(bh.x, ah.x), CFD_N(bh.x, ah.x), out)) nv.x = out;
      if (refresh_value<CASE>(c, nx, ny, j, x.gi + 1, m.y, m.x, Ra, CFD_S(bh.y, ah.y), CFD_N(bh.y, ah.y), out))
        nv.y = out;
    }
    Q[CFD_SLOT(3 + OFF)] = nv;
  }
  {  // residual (+ store) at row A-4d: Q rows A-5d (behind), A-4d, A-3d (ahead)
    const int j = A - 4 * DIR;
    const bool jout = j >= x.y0 && j < x.y1;  // wave-uniform
    if (jout) {
      const double2 m = Q[CFD_SLOT(4 + OFF)], bh = Q[CFD_SLOT(5 + OFF)], ah = Q[CFD_SLOT(3 + OFF)];
      const double Lb = dpp_from_left(m.y), Ra = dpp_from_right(m.x);
      if (store && x.out_lane)
        store_row_pair(x.pout, x.prs, (size_t)(j - x.g.row_lo) * (size_t)x.g.pitch + x.gi, m);
      if (FAST) {
        if (!RC || (j >= x.g.j0 && j <= x.g.j1 && j <= x.res_hi)) {  // row-uniform
          if (CASE == CAVITY && j == ny) {  // top row: eps_n = 0 (cavity-01.cpp:666)
            rm = fmax(rm, residual_abs<CASE>(c, nx, ny, j, x.gi, m.x, Lb, m.y, CFD_S(bh.x, ah.x), CFD_N(bh.x, ah.x), f_res.x));
            rm = fmax(rm, residual_abs<CASE>(c, nx, ny, j, x.gi + 1, m.y, m.x, Ra, CFD_S(bh.y, ah.y), CFD_N(bh.y, ah.y), f_res.y));
          } else {
            // both cells first: results of arithmetic need no canonicalisation,
            // so one max per row touches the loop-carried accumulator
            rm = fmax(rm, fmax(residual_interior<CASE>(c, m.x, Lb, m.y, CFD_S(bh.x, ah.x), CFD_N(bh.x, ah.x), f_res.x),
                               residual_interior<CASE>(c, m.y, m.x, Ra, CFD_S(bh.y, ah.y), CFD_N(bh.y, ah.y), f_res.y)));
          }
        }
      } else if (j >= x.g.j0 && j <= x.g.j1) {
        const double ra =
            residual_abs<CASE>(c, nx, ny, j, x.gi, m.x, Lb, m.y, CFD_S(bh.x, ah.x), CFD_N(bh.x, ah.x), f_res.x);
        const double rb =
            residual_abs<CASE>(c, nx, ny, j, x.gi + 1, m.y, m.x, Ra, CFD_S(bh.y, ah.y), CFD_N(bh.y, ah.y), f_res.y);
        rm = fmax(rm, (x.out_lane && x.fl_a(j)) ? ra : 0.0);
        rm = fmax(rm, (x.out_lane && x.fl_b(j)) ? rb : 0.0);
      }
    }
  }
#undef CFD_S
#undef CFD_N
}

// slot of row R - X*d in a prefetch ring of NPR slots at march step t (t mod
// 10 from ROT = t mod 5 and PAR = t mod 2; NPR == 5 only needs ROT)
#define CFD_NSLOT(X) ((NPR == 5) ? CFD_SLOT(X) : ((((6 * (ROT) + 5 * (PAR)) % 10 + NPR - 1 - (X)) % NPR + 2 * NPR) % NPR))

template <int CASE, int DIR, int ROT, bool FAST, int PAR, int NPR, bool RC = true>  // PAR = parity of R (2: not known at compile time)
__device__ __forceinline__ void wave_pair_step(const WaveCtx<CASE>& x, WavePair<NPR>& s, int R) {
  constexpr int PD = NPR - 1;  // rows in flight ahead of the front row
  static_assert(NPR == 5 || PAR != 2, "deep prefetch rings need the 10-step unroll");
  // consume the prefetched row R (and f row R-d); issue the loads PD rows ahead
  s.fr2[CFD_SLOT(6)] = s.fr[CFD_SLOT(6)];  // f row R-6d leaves fr (its slot takes row R-d) for fr2
  s.w[CFD_SLOT(0)] = s.np[CFD_NSLOT(0)];
  s.fr[CFD_SLOT(1)] = s.nf[CFD_NSLOT(0)];
  if (FAST) {  // rows clamped to stored memory (wave-uniform); out-of-range rows are never consumed
    s.np[CFD_NSLOT(-PD)] = x.ld_fast(x.pin, R + PD * DIR);
    s.nf[CFD_NSLOT(-PD)] = x.ld_fast(x.f, R + (PD - 1) * DIR);
  } else {
    s.np[CFD_NSLOT(-PD)] = x.ld(x.pin, R + PD * DIR);
    s.nf[CFD_NSLOT(-PD)] = x.ld(x.f, R + (PD - 1) * DIR);
  }
  // iteration k: rows R-d .. R-4d
  pair_stages<CASE, DIR, ROT, 0, FAST, PAR, RC>(x, s.w, s.q, s.fr[CFD_SLOT(1)], s.fr[CFD_SLOT(2)], s.fr[CFD_SLOT(4)], R, false,
                                       s.rmax1);
  // iteration k+1 takes iteration k's newest final row (R-3d) as its front row
  s.w2[CFD_SLOT(3)] = s.q[CFD_SLOT(3)];
  pair_stages<CASE, DIR, ROT, 3, FAST, (PAR == 2) ? 2 : (PAR ^ 1), RC>(x, s.w2, s.q2, s.fr[CFD_SLOT(4)], s.fr[CFD_SLOT(5)], s.fr2[CFD_SLOT(7)],
                                       R - 3 * DIR, true, s.rmax2);
}

template <int CASE, int DIR, bool FAST, bool RC = true>
__device__ __forceinline__ void wave_march_pair(const WaveCtx<CASE>& x, int y0, int y1, double& r1, double& r2) {
  constexpr int H = PAIR_H;
  // first front row, moved one row outward if needed so that it is even: the
  // row parity of every stage is then a compile-time constant of the 10-step
  // unrolled loop (no branches on the red/black colour); the extra leading row
  // and the trailing rows of the last 10-step group are pipeline fill only
  // (no store, no residual: outside [y0, y1))
  const int Rb0 = (DIR > 0) ? y0 - H : y1 - 1 + H;
  const int Rbeg = Rb0 - DIR * (Rb0 & 1);
  const int nsteps = (y1 - y0) + 2 * H + (Rb0 & 1);
  constexpr int NPR = FAST ? CFD_PAIR_NPR : 5;
  WavePair<NPR> s;
  const double2 z = make_double2(0.0, 0.0);
#pragma unroll
  for (int k = 0; k < 5; ++k) s.w[k] = s.q[k] = s.w2[k] = s.q2[k] = s.fr[k] = s.fr2[k] = z;
  s.rmax1 = s.rmax2 = 0.0;
  {
    constexpr int ROT = 0, PAR = 0;  // slots as seen by the first step
#pragma unroll
    for (int q = 0; q < NPR - 1; ++q) {
      s.np[CFD_NSLOT(-q)] = FAST ? x.ld_fast(x.pin, Rbeg + q * DIR) : x.ld(x.pin, Rbeg + q * DIR);
      s.nf[CFD_NSLOT(-q)] = FAST ? x.ld_fast(x.f, Rbeg + (q - 1) * DIR) : x.ld(x.f, Rbeg + (q - 1) * DIR);
    }
  }
  int R = Rbeg;
  for (int st = 0; st < nsteps; st += 10, R += 10 * DIR) {
    wave_pair_step<CASE, DIR, 0, FAST, 0, NPR, RC>(x, s, R);
    wave_pair_step<CASE, DIR, 1, FAST, 1, NPR, RC>(x, s, R + DIR);
    wave_pair_step<CASE, DIR, 2, FAST, 0, NPR, RC>(x, s, R + 2 * DIR);
    wave_pair_step<CASE, DIR, 3, FAST, 1, NPR, RC>(x, s, R + 3 * DIR);
    wave_pair_step<CASE, DIR, 4, FAST, 0, NPR, RC>(x, s, R + 4 * DIR);
    wave_pair_step<CASE, DIR, 0, FAST, 1, NPR, RC>(x, s, R + 5 * DIR);
    wave_pair_step<CASE, DIR, 1, FAST, 0, NPR, RC>(x, s, R + 6 * DIR);
    wave_pair_step<CASE, DIR, 2, FAST, 1, NPR, RC>(x, s, R + 7 * DIR);
    wave_pair_step<CASE, DIR, 3, FAST, 0, NPR, RC>(x, s, R + 8 * DIR);
    wave_pair_step<CASE, DIR, 4, FAST, 1, NPR, RC>(x, s, R + 9 * DIR);
  }
  r1 = FAST ? (x.out_lane ? s.rmax1 : 0.0) : s.rmax1;
  r2 = FAST ? (x.out_lane ? s.rmax2 : 0.0) : s.rmax2;
}

// ---- cavity: NS red-black iterations per launch, dependency depth 2NS+1 ----
//
// The cavity has no ghost / solid refresh (its ghosts are fixed zeros), so a
// row is final as soon as its black cells are updated. Sweep s of the launch
// has front row A = R - 2s d: red at A-d, black at A-2d, residual at A-3d;
// row A-2d, final, is the front row of sweep s+1; the last sweep also stores.
// Same operations in the same order per cell as one launch per iteration, so
// the result is bit-identical. NS = 2: 5 halo rows; NS = 3: 7 (the 8-column
// halos of PAIR_TWC fit both). Interior-column waves use the unmasked forms
// (sor_fast / residual_interior, rows by uniform branches); boundary-column
// waves the reference's masked forms (sor_update / residual_abs).

// cavity interior bands march alternately down / up (1), or all down (0)
#ifndef CFD_CAV_UP
#define CFD_CAV_UP 1
#endif
// rows of p_in / f in flight per cavity wave (prefetch distance, <= 9): exact
// launches / proof-mode launches of 3 and 4 sweeps (as deep as 3 waves/SIMD allow)
#ifndef CFD_CAV_PD
#define CFD_CAV_PD 4
#endif
#ifndef CFD_CAV_PD3
#define CFD_CAV_PD3 4
#endif
#ifndef CFD_CAV_PD4
#define CFD_CAV_PD4 4
#endif

template <int NS>
struct CavRun {
  double2 w[NS][5];  // sweep s: rows R-2s d .. R-(2s+4) d
  double2 fr[10];    // source rows R-d .. R-10d
  double2 np[10];    // prefetched p_in rows R .. R+PD d (row R - X d in slot CFD_S10(X))
  double2 nf[10];    // prefetched f rows R-d .. R+(PD-1) d (same slots)
  double rmax[NS];   // exact mode: max |residual| per sweep; proof mode: max |black update| per sweep
  double pm;         // proof mode: max |p_in| over every row this wave loads (all lanes)
};

// ---------------------------------------------- proof-mode convergence test --
//
// The reference keeps sweeping while max|r| > tol (cavity-01.cpp:633, the
// residual of :659-677). To go on it is enough that ONE cell has |r| > tol.
// For a black cell with four neighbours (1 < i < nx, 1 <= j < ny) the
// residual right after its update follows from the update itself: with
// p' = (1-w) p + (w/4) (S - h^2 f) and r = idx2 (S - 4 p') - f,
//     r = K (p' - p) + E,   K = 4 idx2 (1-w)/w,
// where |E| is bounded by the rounding of the update and of the residual's
// own evaluation: |E| + |r_ref - r| <= 128 u idx2 P + 16 u F (u = 2^-53, P a
// bound on every |p| in the cell's stencil, F on |f|; DESIGN.md §2 has the
// derivation; requires 0.5 <= w < 2). Each sweep grows max|p| by at most 9x
// (red then black, w < 2) plus h^2 F, so over a launch P <= 9^NS (Pin + h^2 F),
// Pin = max|p_in| over every value the wave loads (all its cells' cones lie in
// them: no cross-wave or cross-rank bound needed) and F = max|f| over the
// interior (tolerance pass). Hence
//     |p' - p| > thr = (tol + 2^-43 (idx2 P + F)) / |K|  (x (1 + 2^-38))
// proves |r_ref| > tol, i.e. the reference's loop goes on, with the computed
// fields untouched. The wave records max|p' - p| / thr per sweep (> 1:
// proven). A sweep that is not proven this way (only near convergence, or
// with non-finite values) is evaluated exactly: the host reruns the launch
// that computed it with the exact residual kernel and finishes the solve so.
__device__ __forceinline__ double proof_ratio(const Coef& c, double tol, double dmax, double pin, double fmx,
                                              double growth) {
  // (a NaN bound fails every comparison below: q = 0)
  const double P = growth * (pin + c.h2 * fmx) * (1.0 + 0x1p-40);
  const double margin = 0x1p-43 * (c.idx2 * P + fmx);
  const double thr = (tol + margin) / c.proof_k * (1.0 + 0x1p-38);
  const double q = dmax / thr;
  return (q == q && q >= 0.0) ? q : 0.0;  // non-finite bounds prove nothing
}

// slot of row R - X d in a 10-slot ring at step t = (ROT, PAR) of the 10-step march
#define CFD_S10(X) ((((6 * (ROT) + 5 * (PAR)) % 10 + 9 - (X)) % 10 + 20) % 10)

// the lane constants of a cavity boundary-column wave (columns gi, gi+1)
__device__ __forceinline__ void cav_edge_lanes(WaveCtx<CAVITY>& x) {
  const int nx = x.g.nx, ia = x.gi, ib = x.gi + 1;
  x.ce_a = (ia < nx) ? 1.0 : 0.0;
  x.cw_a = (ia > 1) ? 1.0 : 0.0;
  x.ce_b = (ib < nx) ? 1.0 : 0.0;
  x.cw_b = (ib > 1) ? 1.0 : 0.0;
  const int na = (ia < nx) + (ia > 1) + 1, nb = (ib < nx) + (ib > 1) + 1;  // + eps_n (below the top row)
  // om_nc[n] by value: a run-time index into Coef would copy it to scratch
  double o1 = x.c.om_nc[1], o2 = x.c.om_nc[2], o3 = x.c.om_nc[3], o4 = x.c.om_nc[4];
  auto pick = [&](int n) { return n == 4 ? o4 : n == 3 ? o3 : n == 2 ? o2 : o1; };
  x.om_a = pick(na + 1);
  x.om_at = pick(na);
  x.om_b = pick(nb + 1);
  x.om_bt = pick(nb);
}


// red (COLOR 0) / black (COLOR 1) update of row j = R - X d (parity JPAR).
// PROOF (interior waves): the black update also records |p' - p| x wgt
// (wgt = 1 on rows whose cells prove, 0 elsewhere: a row-uniform scalar).
// RC (row checks): the row may be a ghost row or the top row; without them
// (interior bands whose dependency cone stays in rows 1 .. ny-1) every row is
// updated with four neighbours, straight-line code
template <int DIR, int ROT, int JPAR, int COLOR, bool EDGE, bool PROOF = false, bool RC = true>
__device__ __forceinline__ void cav_update(const WaveCtx<CAVITY>& x, double2 (&W)[5], int j, int X,
                                           const double2& fc, double wgt = 0.0, double* dm = nullptr) {
  double2& m = W[CFD_SLOT(X)];
  const double2 bh = W[CFD_SLOT(X + 1)], ah = W[CFD_SLOT(X - 1)];
#define CFD_S(b, a) ((DIR > 0) ? (b) : (a))
#define CFD_N(b, a) ((DIR > 0) ? (a) : (b))
  if (!RC || (j > x.rmin && j < x.rmax)) {  // row-uniform
    if (((JPAR ^ COLOR) & 1) == 0) {  // slot a (even column gi) has this colour
      const double Lb = dpp_from_left(m.y);
      if (EDGE) {
        const double nv = cav_edge_sor(x.c, j == x.g.ny, x.ce_a, x.cw_a, x.om_a, x.om_at, m.x, Lb, m.y,
                                       CFD_S(bh.x, ah.x), CFD_N(bh.x, ah.x), fc.x);
        m.x = x.icol_a ? nv : m.x;  // (the rows here are 1..ny)
      } else {
        const double old = m.x;
        m.x = RC ? sor_fast<CAVITY>(x, j, m.x, Lb, m.y, CFD_S(bh.x, ah.x), CFD_N(bh.x, ah.x), fc.x)
                 : sor_interior<CAVITY>(x.c, m.x, Lb, m.y, CFD_S(bh.x, ah.x), CFD_N(bh.x, ah.x), fc.x);
        if (PROOF && COLOR == 1) *dm = fmax(*dm, fabs(m.x - old) * wgt);
      }
    } else {
      const double Ra = dpp_from_right(m.x);
      if (EDGE) {
        const double nv = cav_edge_sor(x.c, j == x.g.ny, x.ce_b, x.cw_b, x.om_b, x.om_bt, m.y, m.x, Ra,
                                       CFD_S(bh.y, ah.y), CFD_N(bh.y, ah.y), fc.y);
        m.y = x.icol_b ? nv : m.y;
      } else {
        const double old = m.y;
        m.y = RC ? sor_fast<CAVITY>(x, j, m.y, m.x, Ra, CFD_S(bh.y, ah.y), CFD_N(bh.y, ah.y), fc.y)
                 : sor_interior<CAVITY>(x.c, m.y, m.x, Ra, CFD_S(bh.y, ah.y), CFD_N(bh.y, ah.y), fc.y);
        if (PROOF && COLOR == 1) *dm = fmax(*dm, fabs(m.y - old) * wgt);
      }
    }
  }
#undef CFD_S
#undef CFD_N
}

template <int DIR, int ROT, bool EDGE, bool PROOF = false>
__device__ __forceinline__ void cav_residual(const WaveCtx<CAVITY>& x, const double2 (&W)[5], int j, int X,
                                             const double2& fc, bool store, double& rm) {
  const int nx = x.g.nx, ny = x.g.ny;
  const Coef& c = x.c;
#define CFD_S(b, a) ((DIR > 0) ? (b) : (a))
#define CFD_N(b, a) ((DIR > 0) ? (a) : (b))
  if (PROOF) {  // no residual: the store of the last sweep
    (void)rm;
    if (store && j >= x.y0 && j < x.y1 && x.out_lane)
      store_row_pair(x.pout, x.prs, (size_t)(j - x.g.row_lo) * (size_t)x.g.pitch + x.gi, W[CFD_SLOT(X)]);
    return;
  }
  if (j >= x.y0 && j < x.y1) {  // row-uniform
    const double2 m = W[CFD_SLOT(X)], bh = W[CFD_SLOT(X + 1)], ah = W[CFD_SLOT(X - 1)];
    const double Lb = dpp_from_left(m.y), Ra = dpp_from_right(m.x);
    if (store && x.out_lane)
      store_row_pair(x.pout, x.prs, (size_t)(j - x.g.row_lo) * (size_t)x.g.pitch + x.gi, m);
    if (j >= x.g.j0 && j <= x.g.j1) {
      if (EDGE) {
        const bool top = j == ny;
        const double ra = cav_edge_res(c, top, x.ce_a, x.cw_a, m.x, Lb, m.y, CFD_S(bh.x, ah.x), CFD_N(bh.x, ah.x), fc.x);
        const double rb = cav_edge_res(c, top, x.ce_b, x.cw_b, m.y, m.x, Ra, CFD_S(bh.y, ah.y), CFD_N(bh.y, ah.y), fc.y);
        rm = fmax(rm, (x.out_lane && x.icol_a) ? ra : 0.0);  // (rows j0..j1 here)
        rm = fmax(rm, (x.out_lane && x.icol_b) ? rb : 0.0);
      } else if (j == ny) {  // top row: eps_n = 0 (cavity-01.cpp:666)
        rm = fmax(rm, fmax(residual_abs<CAVITY>(c, nx, ny, j, x.gi, m.x, Lb, m.y, CFD_S(bh.x, ah.x), CFD_N(bh.x, ah.x), fc.x),
                           residual_abs<CAVITY>(c, nx, ny, j, x.gi + 1, m.y, m.x, Ra, CFD_S(bh.y, ah.y), CFD_N(bh.y, ah.y), fc.y)));
      } else {
        // both cells first: one max per row touches the loop-carried accumulator
        rm = fmax(rm, fmax(residual_interior<CAVITY>(c, m.x, Lb, m.y, CFD_S(bh.x, ah.x), CFD_N(bh.x, ah.x), fc.x),
                           residual_interior<CAVITY>(c, m.y, m.x, Ra, CFD_S(bh.y, ah.y), CFD_N(bh.y, ah.y), fc.y)));
      }
    }
  }
#undef CFD_S
#undef CFD_N
}

// The first two groups of 10 march steps of an interior wave (GST = the step
// index 0..19 at compile time; p = the parity alignment step, 0 or 1) skip the
// red / black updates of sweep S whose rows lie outside the dependency cone of
// the band's output rows [y0, y1): sweep S is needed on rows
// [y0 - 2(NS-1-S) - 1, ...) (red) and [y0 - 2(NS-1-S), ...) (black), which the
// front reaches at step 3 + 4S + p (red) / 5 + 4S + p (black). Rows outside the
// cone are never read by a needed update (red(S+1) at r reads black(S) at
// r-1..r+1, black(S) reads red(S) likewise), so the stored rows and the proof
// ratios (black rows inside [y0, y1) only) are the same bits (exact-residual
// launches: the residuals of rows [y0, y1) read one row further, so every
// threshold is one step earlier); the skipped
// updates are ~10 % of an interior wave's VALU work (80 of 8 x (th + 19)
// half-row updates at th = 81). The drain end has no such rows: the cone
// reaches past y1 exactly as far as the pipeline lags the front. (cone_step:
// device.hpp)

// sweeps S .. NS-1 of one march step (compile-time recursion over the sweeps)
template <int S, int NS, int DIR, int ROT, int PAR, bool EDGE, bool PROOF, bool RC, int GST = -1>
__device__ __forceinline__ void cav_sweeps(const WaveCtx<CAVITY>& x, CavRun<NS>& s, int R, int p = 0) {
  if constexpr (S < NS) {
    // red at R-(2S+1)d (parity PAR^1), black at R-(2S+2)d (PAR), residual at R-(2S+3)d
    constexpr int sh = PROOF ? 0 : 1;  // (exact residuals of rows [y0, y1) read rows y0-1 / y1: one row more)
    if (cone_step<GST, 3 + 4 * S - sh>(p))
      cav_update<DIR, ROT, PAR ^ 1, 0, EDGE, false, RC>(x, s.w[S], R - (2 * S + 1) * DIR, 2 * S + 1,
                                                        s.fr[CFD_S10(2 * S + 1)]);
    if (cone_step<GST, 5 + 4 * S - sh>(p)) {
      if constexpr (PROOF && !EDGE) {
        const int jb = R - (2 * S + 2) * DIR;
        const double wgt = (jb >= x.py0 && jb < x.py1) ? 1.0 : 0.0;  // row-uniform
        cav_update<DIR, ROT, PAR, 1, EDGE, true, RC>(x, s.w[S], jb, 2 * S + 2, s.fr[CFD_S10(2 * S + 2)], wgt,
                                                     &s.rmax[S]);
      } else {
        cav_update<DIR, ROT, PAR, 1, EDGE, false, RC>(x, s.w[S], R - (2 * S + 2) * DIR, 2 * S + 2,
                                                      s.fr[CFD_S10(2 * S + 2)]);
      }
    }
    cav_residual<DIR, ROT, EDGE, PROOF>(x, s.w[S], R - (2 * S + 3) * DIR, 2 * S + 3, s.fr[CFD_S10(2 * S + 3)],
                                        S == NS - 1, s.rmax[S]);
    if constexpr (S + 1 < NS) s.w[S + 1][CFD_SLOT(2 * S + 2)] = s.w[S][CFD_SLOT(2 * S + 2)];
    cav_sweeps<S + 1, NS, DIR, ROT, PAR, EDGE, PROOF, RC, GST>(x, s, R, p);
  }
}

template <int NS, int DIR, int ROT, int PAR, bool EDGE, bool PROOF, int PD, bool RC, int GST = -1>  // PAR = parity of R
__device__ __forceinline__ void cav_step(const WaveCtx<CAVITY>& x, CavRun<NS>& s, int R, int p = 0) {
  s.w[0][CFD_SLOT(0)] = s.np[CFD_S10(0)];
  s.fr[CFD_S10(1)] = s.nf[CFD_S10(1)];
  if constexpr (PROOF && !EDGE) {  // the proof's Pin: every p_in value this wave uses
    const double2 a = s.np[CFD_S10(0)];
    s.pm = fmax(s.pm, fmax(fabs(a.x), fabs(a.y)));
  }
  if (EDGE) {
    s.np[CFD_S10(-PD)] = x.ld(x.pin, R + PD * DIR);
    s.nf[CFD_S10(1 - PD)] = x.ld(x.f, R + (PD - 1) * DIR);
  } else {
    s.np[CFD_S10(-PD)] = x.ld_fast(x.pin, R + PD * DIR);
    s.nf[CFD_S10(1 - PD)] = x.ld_fast(x.f, R + (PD - 1) * DIR);
  }
  cav_sweeps<0, NS, DIR, ROT, PAR, EDGE, PROOF, RC, GST>(x, s, R, p);
}

// 1: the cavity's proof-mode bands near the top / bottom rows and the
// boundary-column waves run their row groups clear of those rows unchecked
// (measured neutral at 4096^2, 79.3 vs 79.4 us per launch: the cavity's
// launch is balanced - per-wave stamps, profiles/r3_balance/ - so it stays off)
#ifndef CFD_CAV_GROUPS
#define CFD_CAV_GROUPS 0
#endif
// 1: interior waves skip the updates outside their band's dependency cone in
// the first 20 march steps (cav_sweeps)
#ifndef CFD_CAV_CONE
#define CFD_CAV_CONE 1
#endif
// PROOF: r[q] = max |black update| of sweep q over the output cells
// (interior waves; 0 on boundary-column waves), pm = max |p_in| loaded.
// RC: groups of 10 steps whose rows (front, pipeline, neighbours) all lie in
// (gmin, gmax) run without row checks (as open.hip open_march); gmax <= ny
// keeps the top row (eps_n = 0) in the checked steps of interior waves
template <int NS, int DIR, bool EDGE, bool PROOF = false, bool RC = true,
          int PD = !PROOF ? CFD_CAV_PD : (NS == 3) ? CFD_CAV_PD3 : CFD_CAV_PD4>
__device__ __forceinline__ void cav_march(const WaveCtx<CAVITY>& x0, int y0, int y1, double (&r)[NS],
                                          double* pm = nullptr, int gmin = 0, int gmax = 0) {
  WaveCtx<CAVITY> x = x0;
  constexpr int H = 2 * NS + 1;
  const int Rb0 = (DIR > 0) ? y0 - H : y1 - 1 + H;
  const int Rbeg = Rb0 - DIR * (Rb0 & 1);  // even first front row: compile-time colours
  const int nsteps = (y1 - y0) + 2 * H + (Rb0 & 1);
  if constexpr (EDGE) cav_edge_lanes(x);
  CavRun<NS> s;
  const double2 z = make_double2(0.0, 0.0);
#pragma unroll
  for (int k = 0; k < 5; ++k)
#pragma unroll
    for (int q = 0; q < NS; ++q) s.w[q][k] = z;
#pragma unroll
  for (int k = 0; k < 10; ++k) s.fr[k] = z;
#pragma unroll
  for (int q = 0; q < NS; ++q) s.rmax[q] = 0.0;
  s.pm = 0.0;
  {
    constexpr int ROT = 0, PAR = 0;
#pragma unroll
    for (int q = 0; q < PD; ++q) {
      s.np[CFD_S10(-q)] = EDGE ? x.ld(x.pin, Rbeg + q * DIR) : x.ld_fast(x.pin, Rbeg + q * DIR);
      s.nf[CFD_S10(1 - q)] = EDGE ? x.ld(x.f, Rbeg + (q - 1) * DIR) : x.ld_fast(x.f, Rbeg + (q - 1) * DIR);
    }
  }
  int R = Rbeg;
  int st = 0;
#if CFD_CAV_CONE
  if constexpr (!EDGE) {  // the first two groups: updates outside the band's cone skipped (cav_sweeps)
    const int p = Rb0 & 1;
    cav_step<NS, DIR, 0, 0, EDGE, PROOF, PD, RC, 0>(x, s, R, p);
    cav_step<NS, DIR, 1, 1, EDGE, PROOF, PD, RC, 1>(x, s, R + DIR, p);
    cav_step<NS, DIR, 2, 0, EDGE, PROOF, PD, RC, 2>(x, s, R + 2 * DIR, p);
    cav_step<NS, DIR, 3, 1, EDGE, PROOF, PD, RC, 3>(x, s, R + 3 * DIR, p);
    cav_step<NS, DIR, 4, 0, EDGE, PROOF, PD, RC, 4>(x, s, R + 4 * DIR, p);
    cav_step<NS, DIR, 0, 1, EDGE, PROOF, PD, RC, 5>(x, s, R + 5 * DIR, p);
    cav_step<NS, DIR, 1, 0, EDGE, PROOF, PD, RC, 6>(x, s, R + 6 * DIR, p);
    cav_step<NS, DIR, 2, 1, EDGE, PROOF, PD, RC, 7>(x, s, R + 7 * DIR, p);
    cav_step<NS, DIR, 3, 0, EDGE, PROOF, PD, RC, 8>(x, s, R + 8 * DIR, p);
    cav_step<NS, DIR, 4, 1, EDGE, PROOF, PD, RC, 9>(x, s, R + 9 * DIR, p);
    st += 10;
    R += 10 * DIR;
    if (nsteps > 10) {
      cav_step<NS, DIR, 0, 0, EDGE, PROOF, PD, RC, 10>(x, s, R, p);
      cav_step<NS, DIR, 1, 1, EDGE, PROOF, PD, RC, 11>(x, s, R + DIR, p);
      cav_step<NS, DIR, 2, 0, EDGE, PROOF, PD, RC, 12>(x, s, R + 2 * DIR, p);
      cav_step<NS, DIR, 3, 1, EDGE, PROOF, PD, RC, 13>(x, s, R + 3 * DIR, p);
      cav_step<NS, DIR, 4, 0, EDGE, PROOF, PD, RC, 14>(x, s, R + 4 * DIR, p);
      cav_step<NS, DIR, 0, 1, EDGE, PROOF, PD, RC, 15>(x, s, R + 5 * DIR, p);
      cav_step<NS, DIR, 1, 0, EDGE, PROOF, PD, RC, 16>(x, s, R + 6 * DIR, p);
      cav_step<NS, DIR, 2, 1, EDGE, PROOF, PD, RC, 17>(x, s, R + 7 * DIR, p);
      cav_step<NS, DIR, 3, 0, EDGE, PROOF, PD, RC, 18>(x, s, R + 8 * DIR, p);
      cav_step<NS, DIR, 4, 1, EDGE, PROOF, PD, RC, 19>(x, s, R + 9 * DIR, p);
      st += 10;
      R += 10 * DIR;
    }
  }
#endif
  constexpr int BACK = 2 * NS + 5;  // rows behind the front a step touches (+1)
  for (; st < nsteps; st += 10, R += 10 * DIR) {
#if CFD_CAV_GROUPS
    const int glo = (DIR > 0) ? R - BACK : R - 11, ghi = (DIR > 0) ? R + 11 : R + BACK;
    if (RC && glo > gmin && ghi < gmax) {  // (wave-uniform)
      cav_step<NS, DIR, 0, 0, EDGE, PROOF, PD, false>(x, s, R);
      cav_step<NS, DIR, 1, 1, EDGE, PROOF, PD, false>(x, s, R + DIR);
      cav_step<NS, DIR, 2, 0, EDGE, PROOF, PD, false>(x, s, R + 2 * DIR);
      cav_step<NS, DIR, 3, 1, EDGE, PROOF, PD, false>(x, s, R + 3 * DIR);
      cav_step<NS, DIR, 4, 0, EDGE, PROOF, PD, false>(x, s, R + 4 * DIR);
      cav_step<NS, DIR, 0, 1, EDGE, PROOF, PD, false>(x, s, R + 5 * DIR);
      cav_step<NS, DIR, 1, 0, EDGE, PROOF, PD, false>(x, s, R + 6 * DIR);
      cav_step<NS, DIR, 2, 1, EDGE, PROOF, PD, false>(x, s, R + 7 * DIR);
      cav_step<NS, DIR, 3, 0, EDGE, PROOF, PD, false>(x, s, R + 8 * DIR);
      cav_step<NS, DIR, 4, 1, EDGE, PROOF, PD, false>(x, s, R + 9 * DIR);
      continue;
    }
#else
    (void)gmin;
    (void)gmax;
    (void)BACK;
#endif
    cav_step<NS, DIR, 0, 0, EDGE, PROOF, PD, RC>(x, s, R);
    cav_step<NS, DIR, 1, 1, EDGE, PROOF, PD, RC>(x, s, R + DIR);
    cav_step<NS, DIR, 2, 0, EDGE, PROOF, PD, RC>(x, s, R + 2 * DIR);
    cav_step<NS, DIR, 3, 1, EDGE, PROOF, PD, RC>(x, s, R + 3 * DIR);
    cav_step<NS, DIR, 4, 0, EDGE, PROOF, PD, RC>(x, s, R + 4 * DIR);
    cav_step<NS, DIR, 0, 1, EDGE, PROOF, PD, RC>(x, s, R + 5 * DIR);
    cav_step<NS, DIR, 1, 0, EDGE, PROOF, PD, RC>(x, s, R + 6 * DIR);
    cav_step<NS, DIR, 2, 1, EDGE, PROOF, PD, RC>(x, s, R + 7 * DIR);
    cav_step<NS, DIR, 3, 0, EDGE, PROOF, PD, RC>(x, s, R + 8 * DIR);
    cav_step<NS, DIR, 4, 1, EDGE, PROOF, PD, RC>(x, s, R + 9 * DIR);
  }
  if constexpr (PROOF) {
    *pm = s.pm;
#pragma unroll
    for (int q = 0; q < NS; ++q) r[q] = (!EDGE && x.out_lane) ? s.rmax[q] : 0.0;
  } else {
#pragma unroll
    for (int q = 0; q < NS; ++q) r[q] = (EDGE || x.out_lane) ? s.rmax[q] : 0.0;
  }
}
#undef CFD_S10

// Boundary-column waves (ghost / solid columns in the tile): general masks
// and a 5-step unroll with the colour tested at run time - compact code, so
// that it shares the instruction cache with the interior loops.
template <int CASE, int DIR>
__device__ __forceinline__ void wave_march_pair_edge(const WaveCtx<CASE>& x, int y0, int y1, double& r1,
                                                     double& r2) {
  constexpr int H = PAIR_H;
  const int Rbeg = (DIR > 0) ? y0 - H : y1 - 1 + H;
  const int nsteps = (y1 - y0) + 2 * H;
  constexpr int NPR = 5;
  WavePair<NPR> s;
  const double2 z = make_double2(0.0, 0.0);
#pragma unroll
  for (int k = 0; k < 5; ++k) s.w[k] = s.q[k] = s.w2[k] = s.q2[k] = s.fr[k] = s.fr2[k] = z;
  s.rmax1 = s.rmax2 = 0.0;
  {
    constexpr int ROT = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      s.np[CFD_SLOT(-q)] = x.ld(x.pin, Rbeg + q * DIR);
      s.nf[CFD_SLOT(-q)] = x.ld(x.f, Rbeg + (q - 1) * DIR);
    }
  }
  int st = 0, R = Rbeg;
  for (; st + 5 <= nsteps; st += 5, R += 5 * DIR) {
    wave_pair_step<CASE, DIR, 0, false, 2, 5>(x, s, R);
    wave_pair_step<CASE, DIR, 1, false, 2, 5>(x, s, R + DIR);
    wave_pair_step<CASE, DIR, 2, false, 2, 5>(x, s, R + 2 * DIR);
    wave_pair_step<CASE, DIR, 3, false, 2, 5>(x, s, R + 3 * DIR);
    wave_pair_step<CASE, DIR, 4, false, 2, 5>(x, s, R + 4 * DIR);
  }
  if (st < nsteps) { wave_pair_step<CASE, DIR, 0, false, 2, 5>(x, s, R); ++st; R += DIR; }
  if (st < nsteps) { wave_pair_step<CASE, DIR, 1, false, 2, 5>(x, s, R); ++st; R += DIR; }
  if (st < nsteps) { wave_pair_step<CASE, DIR, 2, false, 2, 5>(x, s, R); ++st; R += DIR; }
  if (st < nsteps) { wave_pair_step<CASE, DIR, 3, false, 2, 5>(x, s, R); ++st; R += DIR; }
  r1 = s.rmax1;
  r2 = s.rmax2;
}
#undef CFD_NSLOT
#undef CFD_SLOT

#ifndef CFD_PAIR_MIN_WAVES
#define CFD_PAIR_MIN_WAVES 2
#endif
#ifndef CFD_CAV_MIN_WAVES
#define CFD_CAV_MIN_WAVES 3  // the cavity pair kernel fits 3 waves/SIMD with room (129 VGPRs)
#endif

// Tiling of one pair launch. Rows are covered in up to two ranges [lo0, hi0)
// and [lo1, hi1) (the second may be empty): one launch for a whole strip, or,
// on ranks that overlap the halo exchange, one launch for the interior rows
// and one for the rows next to both neighbours. Every column tile splits each
// range into bands; the first and last column tile (boundary columns, masked
// march) use shorter bands of `the` rows.
struct PairPlan {
  int ctiles;
  int th, nb0, nb1;    // interior column tiles: band height, bands in range 0 / 1
  int the, nbe0, nbe1; // boundary column tiles
  int lo0, hi0, lo1, hi1;
  int cxa, cxb;        // step: column tiles across the step's column (+1; 0: none), banded like the boundary ones
  // step, proof launches (open.hip) only: the block's column tiles. Tiles
  // 1..nl lie left of the step's column, tiles nl+1..nl+ncx cross it (then
  // cxa = cxb = 0: not boundary-class). Below the block, for both: nlf bands
  // of th rows over [lo0, lz) march the interior-column path (away from the
  // block edge), nle bands of `the` rows over [lz, le) the masked one, le =
  // inlet_jmax + 2 (the block's lower edge row included). Above: the left
  // tiles' nlt bands of `the` rows over [lt, hi0) when the range holds ghost
  // row ny + 1 (refreshed from the block's top row; the block's interior rows
  // between never change, both buffers hold them), the crossing tiles' nxt
  // bands over [le, hi0) (fluid right of the block). ncx = 0: no such class.
  int nl, ncx, nlf, nle, nlt, nxt, lz, le, lt;
  // step, reference-order steady launches (lexw.hpp): the crossing column
  // tiles xa .. xa + xn - 1 march their bands xb .. xb + xbn - 1 (those that
  // reach the block's edge: the per-cell solid rules, ~1.7x the cycles per
  // row) as xparts shorter bands, the extra parts' waves after the interior ones
  int xa, xn, xb, xbn, xparts;
};

// column tiles banded as boundary tiles (masked march): the first and last,
// and the step's mixed ones
__host__ __device__ inline int plan_edge_tiles(const PairPlan& pl) {
  return (pl.ctiles >= 2 ? 2 : 1) + (pl.cxa > 0) + (pl.cxb > 0);
}

// waves of a plan (every class)
__host__ __device__ inline int plan_waves(const PairPlan& pl) {
  const int ne = plan_edge_tiles(pl);
  return ne * (pl.nbe0 + pl.nbe1) + pl.nl * (pl.nlf + pl.nle + pl.nlt) + pl.ncx * (pl.nlf + pl.nle + pl.nxt) +
         (pl.ctiles - ne - pl.nl - pl.ncx) * (pl.nb0 + pl.nb1);
}

// PROOF (cavity): the convergence test of each sweep is the proof above
// instead of the max-norm residual; the fields are the same bits.
#ifndef CFD_PROOF_MIN_WAVES
#define CFD_PROOF_MIN_WAVES 2  // proof-mode launches are planned for 2 waves per SIMD (Solver::init)
#endif
// diagnostic build only (CFD_MARCH_STAMPS=1, never the product library): each
// wave's march cycles with its tile, band and path (solver.hip cfd_march_stamps)
#ifndef CFD_MARCH_STAMPS
#define CFD_MARCH_STAMPS 0
#endif
#if CFD_MARCH_STAMPS
constexpr int MARCH_STAMP_MAX = 8192;
static __device__ long long march_stamp_buf[MARCH_STAMP_MAX * 8];
#endif

template <int CASE, int NS, bool PROOF = false>
__global__ __launch_bounds__(256, PROOF ? CFD_PROOF_MIN_WAVES : (CASE == CAVITY) ? CFD_CAV_MIN_WAVES : CFD_PAIR_MIN_WAVES) void poisson_multi_kernel(
    Geo g, Coef c, const double* __restrict__ pin, double* __restrict__ pout, const double* __restrict__ f,
    PoissonCtl ctl, int k, int ka, int kb, PairPlan pl, int flags) {
  // NS red-black iterations k .. k+NS-1 in one launch (NS = 3: cavity only)
  // (NS = 4: proof mode only - without the residual stage its dependency depth
  // is 2 NS = 8 rows / columns, the stored halo)
  static_assert(NS == 2 || (NS == 3 && CASE == CAVITY) || (NS == 4 && PROOF), "sweeps per launch");
  static_assert(!PROOF || CASE == CAVITY, "proof-mode test: cavity pipeline only");
  // tiles: the first and last column tile (boundary columns, general masks)
  // in bands of pl.the rows, then the interior column tiles in bands of pl.th
  // rows; the host makes the boundary bands shorter so that their slower
  // march ends with the others (one resident round)
  constexpr int H = 8;  // column halo (lanes 0-3 and 60-63)
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: band / row logic stays scalar

  // convergence test of the iterations [ka, kb] (flags bit 2: none, a replay)
  if (!(flags & 4) && !window_go_on(ctl, ka, kb, lane, blockIdx.x == 0 && wv == 0, (flags & 128) != 0)) return;
  if (blockIdx.x == 0 && wv == 0 && lane < RES_SHARDS) {
    // the next launch's residual slots: RING_AHEAD of them whatever this
    // launch's sweep count, because the next launch may run more sweeps than
    // this one (an exact 3-sweep launch followed by a 4-sweep proof-mode launch
    // after a fallback): a slot it atomically maxes into must start at zero
#pragma unroll
    for (int q = 0; q < RING_AHEAD; ++q)
      ctl.ring[(size_t)((k + NS + q) & (RING - 1)) * RES_SHARDS * SHARD_STRIDE + lane * SHARD_STRIDE] = 0.0;
  }

  const int nblk = (int)gridDim.x;
  const int L8 = (nblk / 8) * 8;
  const int bl = (int)blockIdx.x;
  const int blk = ((flags & 2) && bl < L8) ? (bl % 8) * (nblk / 8) + bl / 8 : bl;
  const int tile = blk * 4 + wv;
  const int ne = (pl.ctiles >= 2) ? 2 : 1;
  const int ned = plan_edge_tiles(pl);
  const int nbe = pl.nbe0 + pl.nbe1, nbi = pl.nb0 + pl.nb1;
  int band, ctile, th, nb0;
  if (tile < ned * nbe) {
    const int e = tile / nbe;  // boundary tiles 0 / last, then the step's mixed ones
    ctile = (e == 0) ? 0 : (e == 1 && ne == 2) ? pl.ctiles - 1 : (e == ne && pl.cxa > 0) ? pl.cxa - 1 : pl.cxb - 1;
    band = tile % nbe;
    th = pl.the;
    nb0 = pl.nbe0;
  } else {
    const int t = tile - ned * nbe;
    const int nci = pl.ctiles - ned;
    if (t >= nci * nbi) return;
    // column tiles of one band side by side: their shared halo columns are
    // read at the same moment on the same XCD (one L2); flags bit 3: the bands
    // of one column tile one after another instead (their shared halo rows on
    // one XCD)
    if (flags & 8) {
      ctile = 1 + t / nbi;
      band = t % nbi;
    } else {
      ctile = 1 + t % nci;
      band = t / nci;
    }
    // skip the mixed tiles (cxa < cxb, both inside 1 .. ctiles-2)
    if (pl.cxa > 0 && ctile >= pl.cxa - 1) ++ctile;
    if (pl.cxb > 0 && ctile >= pl.cxb - 1) ++ctile;
    th = pl.th;
    nb0 = pl.nb0;
  }
  const int gi = ctile * PAIR_TWC - H + 2 * lane;
  const bool r0 = band < nb0;
  const int y0 = r0 ? pl.lo0 + band * th : pl.lo1 + (band - nb0) * th;
  const int y1 = min(y0 + th, r0 ? pl.hi0 : pl.hi1);
  if (y0 >= y1) return;
  WaveCtx<CASE> x{g, c};
  x.pin = pin; x.pout = pout; x.f = f;
  x.prs = out_rsrc(pout, g);
  x.gi = gi;
  x.y0 = y0;
  x.y1 = y1;
  x.rmin = max(g.row_lo, 0);
  x.rmax = min(g.row_lo + g.nrows - 1, g.ny + 1);
  x.pair_ok = gi >= 0 && gi + 1 < g.pitch;
  x.out_lane = x.pair_ok && lane >= H / 2 && lane < 64 - H / 2;
  x.icol_a = gi >= 1 && gi <= g.nx;
  x.icol_b = gi + 1 >= 1 && gi + 1 <= g.nx;
  x.open_a = (CASE != BACKSTEP) || (gi > c.step_i);
  x.open_b = (CASE != BACKSTEP) || (gi + 1 > c.step_i);
  x.gic = min(max(gi, 0), g.pitch - 2);
  // interior-column wave: all 128 columns are fluid cells with fluid
  // neighbours (rows are handled row-uniformly inside the fast march)
  const int c0 = ctile * PAIR_TWC - H;
  bool cols_in = c0 >= 1 && c0 + 127 <= g.nx && (CASE != BACKSTEP || c0 > c.step_i + 1);
  if (CASE == BACKSTEP && c0 >= 1 && c0 + 127 <= g.nx && !cols_in) {
    // column tiles over the solid block (i <= step_i, j > inlet_jmax): a band
    // whose march (rows y0-10 .. y1+10 cover the pipeline and its neighbours)
    // stays below the block is plain fluid (interior path); one that stays
    // inside the block, away from fluid and from ghost rows, is never updated
    // or refreshed (both buffers hold its values): nothing to do
    if (y1 + 10 <= c.inlet_jmax - 1) cols_in = true;
    else if (y0 - 10 >= c.inlet_jmax + 2 && y1 + 10 <= g.ny && c0 + 128 <= c.step_i - 1) return;
    else if (c0 + 128 <= c.step_i - 1 && y0 - 10 >= 1 && y1 + 10 <= g.ny) {
      // a band across the block's lower edge, every column inside the block:
      // fluid below, solid above, row-uniform - the interior path with the
      // edge row rules (WaveCtx uhi / blk_row / res_hi), not per-cell masks
      cols_in = true;
      x.uhi = c.inlet_jmax + 1;
      x.blk_row = c.inlet_jmax + 1;
      x.res_hi = c.inlet_jmax;
    }
  }
  const bool up = CFD_CAV_UP && (flags & 1) && (band & 1);
  // interior band whose march (rows y0 - 2NS - 2 .. y1 + 2NS + 1: the
  // dependency cone and the pipeline's own rows) stays inside rows 1 .. ny-1:
  // no row checks (cav_update RC)
  const bool safe = y0 - (2 * NS + 2) > x.rmin && y1 + (2 * NS + 2) < min(x.rmax, g.ny);
  const bool fast = cols_in;
#if CFD_MARCH_STAMPS
  long long t0_;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0_)::"memory");
#endif
  double r[NS];
  if constexpr (CASE == CAVITY) {  // the cavity's own pipeline (no refresh stage: depth 2NS+1)
    if constexpr (PROOF) {
      x.py0 = max(y0, 1);
      x.py1 = min(y1, g.ny);
      double pm = 0.0;
      const int gmin = x.rmin, gmax = min(x.rmax, g.ny);  // (cav_march: unchecked row groups)
      if (!fast) cav_march<NS, 1, true, true>(x, y0, y1, r, &pm, gmin, gmax);
      else if (safe && up) cav_march<NS, -1, false, true, false>(x, y0, y1, r, &pm);
      else if (safe) cav_march<NS, 1, false, true, false>(x, y0, y1, r, &pm);
      else if (up) cav_march<NS, -1, false, true>(x, y0, y1, r, &pm, gmin, gmax);
      else cav_march<NS, 1, false, true>(x, y0, y1, r, &pm, gmin, gmax);
      // P bound: this wave's own max|p_in| (its cells' cones lie in what it
      // loaded), grown over the launch's sweeps
      constexpr double growth = (NS == 2) ? 81.0 : (NS == 3) ? 729.0 : 6561.0;
      const double pin = wave_max(pm), F = ctl.tol[2], tol = ctl.tol[0];
#pragma unroll
      for (int q = 0; q < NS; ++q) r[q] = proof_ratio(c, tol, wave_max(r[q]), pin, F, growth);
    } else {
      if (!fast) cav_march<NS, 1, true>(x, y0, y1, r);
      else if (safe && up) cav_march<NS, -1, false, false, false>(x, y0, y1, r);
      else if (safe) cav_march<NS, 1, false, false, false>(x, y0, y1, r);
      else if (up) cav_march<NS, -1, false>(x, y0, y1, r);
      else cav_march<NS, 1, false>(x, y0, y1, r);
    }
  } else {
    double r1 = 0.0, r2 = 0.0;
    if (fast) {
      // bands whose march (rows y0 - 9 .. y1 + 8) stays off the ghost rows:
      // no row checks, no refresh
      const bool osafe = x.blk_row < 0 && y0 - (PAIR_H + 2) > x.rmin && y1 + (PAIR_H + 2) < min(x.rmax, g.ny + 1);
      if (osafe && up) wave_march_pair<CASE, -1, true, false>(x, y0, y1, r1, r2);
      else if (osafe) wave_march_pair<CASE, 1, true, false>(x, y0, y1, r1, r2);
      else if (up) wave_march_pair<CASE, -1, true>(x, y0, y1, r1, r2);
      else wave_march_pair<CASE, 1, true>(x, y0, y1, r1, r2);
    } else {  // boundary-column waves march one way (compact code)
      wave_march_pair_edge<CASE, 1>(x, y0, y1, r1, r2);
    }
    r[0] = r1;
    r[NS - 1] = r2;
  }
#pragma unroll
  for (int q = 0; q < NS; ++q) r[q] = wave_max(r[q]);
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      double* sl = ctl.ring + (size_t)((k + q) & (RING - 1)) * RES_SHARDS * SHARD_STRIDE;
      atomicMax(reinterpret_cast<unsigned long long*>(sl + (size_t)(tile % RES_SHARDS) * SHARD_STRIDE),
                (unsigned long long)__double_as_longlong(r[q]));
    }
  }
#if CFD_MARCH_STAMPS
  {
    long long t1_;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1_)::"memory");
    if (tile < MARCH_STAMP_MAX && lane < 8) {
      const long long v[8] = {tile, ctile, band, y0, y1, fast ? 1 : 0, safe ? 1 : 0, t1_ - t0_};
      long long o = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) o = lane == q ? v[q] : o;
      march_stamp_buf[(size_t)tile * 8 + lane] = o;
    }
  }
#endif
}

}  // namespace cfd
