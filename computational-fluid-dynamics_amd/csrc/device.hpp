// device.hpp — types and device helpers shared by the SOR kernels of
// kernels.hpp, lexw.hpp, small.hpp and tile.hip: inline / template
// functions only, no kernels, so several translation units may include it.
//
// Layout: each field of a strip is a row-major slab of
// `nrows` x `pitch` doubles; global cell (j, i) lives at
// (j - row_lo) * pitch + i. Row 0 / ny+1 and column 0 / nx+1 are the
// reference's ghost layers; a strip additionally stores HALO rows of its
// neighbours on each side.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cfd {

constexpr int CAVITY = 0, CHANNEL = 1, BACKSTEP = 2;
#ifndef CFD_WAVE_MIN_WAVES
#define CFD_WAVE_MIN_WAVES 3  // waves per SIMD the SOR wave kernel must fit (4 would cap VGPRs at 128 and spill)
#endif
constexpr int HALO = 8;           // halo rows stored per side (a fused pair of SOR iterations needs 7)
constexpr int RES_SHARDS = 32;    // residual / max accumulators, one 128-B line each
constexpr int SHARD_STRIDE = 16;  // doubles between shards (128 B)
constexpr int RING = 16;          // residual ring slots (iteration k uses k & 15)
// Slots a launch of iterations k..k+NS-1 clears for the next launch: k+NS ..
// k+NS+RING_AHEAD-1, as many as the longest launch (4 sweeps). The farthest,
// k+NS+3 = k+NS+3-16 mod RING, lies below every slot still read: the tested
// window (at most two launches back, >= k-8) and this launch's own.
constexpr int RING_AHEAD = 4;
static_assert(4 + RING_AHEAD + 8 <= RING, "ring too small for the tested window and the cleared slots");

struct Geo {
  int nx, ny;      // global interior cells
  int pitch;       // doubles per stored row
  int row_lo;      // global row index of stored row 0
  int nrows;       // stored rows
  int j0, j1;      // owned interior rows (global, inclusive)
  int wj0, wj1;    // owned rows incl. physical ghost rows on boundary strips
};

struct Coef {
  int case_id;
  int step_i, inlet_jmax;  // backwards step: solid block is i <= step_i, j > inlet_jmax
  double dx, dy;
  double idx, idy, idx2, idy2;  // 1/dx, 1/dy, 1/(dx*dx), 1/(dy*dy)
  double nu, dt, rho, u_ref;
  double omega;
  double one_m_omega;      // 1.0 - omega (same rounding as the reference's expression)
  double om_nc[5];         // cavity: omega / neighbour_count for counts 0..4
  double h2;               // cavity: grid_spacing * grid_spacing
  double denom;            // open cases: 2*(idx2+idy2)
  double rdenom;           // open cases: 1.0 / denom (correctly rounded, host)
  double rdenom_lo;        // open cases: RN((1 - rdenom*denom) / denom): rdenom + rdenom_lo ~ 1/denom to 2^-106
  double cav_src;          // cavity: (1/dt) * rho           (cavity-01.cpp:624)
  double open_src;         // open:   rho / dt               (channel-01.cpp:610)
  double cav_corr;         // cavity: (dt/h) * rho           (cavity-01.cpp:696,701)
  double open_cu, open_cv; // open:   dt/(rho*dx), dt/(rho*dy) (channel-01.cpp:697,701)
  double tol_factor, abs_tol;
  double proof_k;          // proof-mode test: |K| = d |1-omega| / omega, d = 4 idx2 (cavity) or denom (open
                           // cases): a black cell's residual is K (p' - p) + rounding (0: test unavailable)
  // Rayleigh-Benard (runs as case CAVITY with the lid at rest, plus T)
  double kappa, buoy, t_hot, t_cold, t_ref;
  // proof-mode bounds (tile.hip tile_proof_ratio): margin 2^-43 (proof_pm P + F),
  // per-sweep growth of P + proof_fd F: cavity idx2 / h2, open cases denom / 1/denom
  double proof_pm, proof_fd;
};

// Control block for one Poisson solve (device memory).
struct PoissonCtl {
  double* ring;        // RING x RES_SHARDS x SHARD_STRIDE residual accumulators
  const double* tol;   // [0] tolerance, [1] initial residual, [2] max|source| (set by tol_kernel)
  int* stop;           // [0] converged flag, [1] iteration count at convergence
  int check_every;
};

__device__ __forceinline__ size_t at(const Geo& g, int j, int i) {
  return (size_t)(j - g.row_lo) * (size_t)g.pitch + (size_t)i;
}

// backwards_step-01.cpp:492-520 (analytic mask: solid block upstream of the
// step above the inlet channel); cavity / channel: every interior cell fluid.
__device__ __forceinline__ bool is_fluid(const Coef& c, int nx, int ny, int j, int i) {
  if (i < 1 || i > nx || j < 1 || j > ny) return false;
  if (c.case_id != BACKSTEP) return true;
  return (i > c.step_i) || (j <= c.inlet_jmax);
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Block-wide max of non-negative values -> one atomicMax on a shard.
template <int NT>
__device__ __forceinline__ void block_max_to_shard(double v, double* shards, int shard) {
  __shared__ double red[NT / 64];
  v = wave_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double m = red[0];
#pragma unroll
    for (int k = 1; k < NT / 64; ++k) m = fmax(m, red[k]);
    // Non-negative doubles order like their bit patterns.
    atomicMax(reinterpret_cast<unsigned long long*>(shards + (size_t)shard * SHARD_STRIDE),
              (unsigned long long)__double_as_longlong(m));
  }
}

// Deterministic block sum (fixed butterfly + fixed wave order).
template <int NT>
__device__ __forceinline__ double block_sum(double v) {
  __shared__ double red[NT / 64];
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0) {
    s = red[0];
#pragma unroll
    for (int k = 1; k < NT / 64; ++k) s += red[k];
  }
  return s;  // valid in thread 0
}

// Row neighbours across lanes (wave shifts).
// bound_ctrl: the lane without a source (0 resp. 63) reads 0, with no
// zero-initialised destination to merge into (one v_mov_dpp per dword)
__device__ __forceinline__ double dpp_from_left(double v) {  // lane l receives lane l-1 (wave_shr:1)
  int lo = __double2loint(v), hi = __double2hiint(v);
  lo = __builtin_amdgcn_mov_dpp(lo, 0x138, 0xf, 0xf, true);
  hi = __builtin_amdgcn_mov_dpp(hi, 0x138, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double dpp_from_right(double v) {  // lane l receives lane l+1 (wave_shl:1)
  int lo = __double2loint(v), hi = __double2hiint(v);
  lo = __builtin_amdgcn_mov_dpp(lo, 0x130, 0xf, 0xf, true);
  hi = __builtin_amdgcn_mov_dpp(hi, 0x130, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}

// ------------------------------------------------------------- Poisson --
//
// Red-black SOR of the reference's pressure equation. Each launch reads p_in
// and f once and writes p_out once (24 B per cell) for one or several fused
// iterations (below); p_in / p_out ping-pong, so tiles never read a
// neighbour's new values and overlapping halos are recomputed redundantly.
//
// SOR updates: cavity-01.cpp:643-654 (indicator form), channel-01.cpp:659-666
// / backwards_step-01.cpp:900-909 (anisotropic form). Residuals:
// cavity-01.cpp:659-677, channel-01.cpp:672-681, backwards_step-01.cpp:916-930.
// Ghost / solid refresh after each sweep: channel-01.cpp:531-541,
// backwards_step-01.cpp:685-740.

// x / denom, correctly rounded, without the divide sequence. y = RN(1/denom)
// and ylo = RN((1 - y*denom)/denom) (host; 1 - y*denom is exact), so y + ylo
// is 1/denom to ~2^-106 relative: q0 = RN(x*y + RN(x*ylo)) is within 2^-105
// relative of x/denom before its rounding, hence a faithful quotient. One FMA
// correction q = RN(q0 + RN(x - q0*denom)*y) (the residual is exact in an FMA
// for a faithful q0) then returns RN(x/denom) by Markstein's theorem (y has
// relative error below 2^-53). Four operations; the former form (q0 = RN(x*y)
// and two corrections) took five. denom > 0, so the quotient has x's sign
// (the copysign keeps -0/denom = -0, which the correction turns into +0).
// Finite, normal operands (pressure sums): no over/underflow. Checked against
// the IEEE divide in tests/test_division.py (random and adversarial
// denominators, quotients next to rounding midpoints).
__device__ __forceinline__ double div_denom(const Coef& c, double x) {
  const double d = c.denom, y = c.rdenom;
  double q = fma(x, y, x * c.rdenom_lo);
  q = fma(fma(-q, d, x), y, q);
  return copysign(q, x);
}

template <int CASE>
__device__ __forceinline__ double sor_update(const Coef& c, int nx, int ny, int j, int i, double pc, double pW,
                                             double pE, double pS, double pN, double fc) {
  if (CASE == CAVITY) {
    const int ew = (i > 1) ? 1 : 0;
    const int ee = (i < nx) ? 1 : 0;
    const int en = (j < ny) ? 1 : 0;
    const int es = 1;
    const int nc = ew + ee + en + es;
    // c.om_nc[nc] == c.omega / nc and c.one_m_omega == 1.0 - c.omega, computed once on the host.
    // Indicator products without int->double multiplies: 1*x == x and, for
    // finite x, 0*x == copysign(0, x) — the same bits as the reference's product.
    const double tE = ee ? pE : copysign(0.0, pE);
    const double tW = ew ? pW : copysign(0.0, pW);
    const double tN = en ? pN : copysign(0.0, pN);
    // selected as values: a run-time index into Coef (or a select of its
    // addresses, which the optimiser forms from a select of loads) copies the
    // whole struct to scratch; the empty asm keeps the loaded values opaque
    double o1 = c.om_nc[1], o2 = c.om_nc[2], o3 = c.om_nc[3], o4 = c.om_nc[4];
    asm("" : "+s"(o1), "+s"(o2), "+s"(o3), "+s"(o4));
    const double om = (nc == 4) ? o4 : (nc == 3) ? o3 : (nc == 2) ? o2 : o1;
    return pc * c.one_m_omega + om * ((tE + tW) + (tN + pS) - fc * c.h2);
  } else {
    const double sum = c.idx2 * (pE + pW) + c.idy2 * (pN + pS);
    const double gs = div_denom(c, sum - fc);  // (sum - fc) / denom
    return c.one_m_omega * pc + c.omega * gs;
  }
}

template <int CASE>
__device__ __forceinline__ double residual_at(const Coef& c, int nx, int ny, int j, int i, double pc, double pW,
                                              double pE, double pS, double pN, double fc) {
  if (CASE == CAVITY) {
    const int ew = (i > 1) ? 1 : 0, ee = (i < nx) ? 1 : 0, en = (j < ny) ? 1 : 0, es = 1;
    const double ih2 = c.idx2;
    return ih2 * (ee * (pE - pc) + ew * (pW - pc) + en * (pN - pc) + es * (pS - pc)) - fc;
  } else {
    const double lap = (pE - 2.0 * pc + pW) * c.idx2 + (pN - 2.0 * pc + pS) * c.idy2;
    return lap - fc;
  }
}

template <int CASE>
__device__ __forceinline__ bool refresh_value(const Coef& c, int nx, int ny, int gj, int gi, double self,
                                              double pW, double pE, double pS, double pN, double& out) {
  // channel-01.cpp:531-541, backwards_step-01.cpp:685-740 (pre-refresh neighbour values)
  if (CASE == CAVITY) return false;
  const bool jin = gj >= 1 && gj <= ny, iin = gi >= 1 && gi <= nx;
  if (gi == 0 && jin) { out = pE; return true; }
  if (gi == nx + 1 && jin) { out = 0.0; return true; }
  if (gj == 0 && iin) { out = pN; return true; }
  if (gj == ny + 1 && iin) { out = pS; return true; }
  if (CASE == BACKSTEP && jin && iin && !is_fluid(c, nx, ny, gj, gi)) {
    double sum = 0.0;
    int n = 0;
    if (gi > 1 && is_fluid(c, nx, ny, gj, gi - 1)) { sum += pW; n++; }
    if (gi < nx && is_fluid(c, nx, ny, gj, gi + 1)) { sum += pE; n++; }
    if (gj > 1 && is_fluid(c, nx, ny, gj - 1, gi)) { sum += pS; n++; }
    if (gj < ny && is_fluid(c, nx, ny, gj + 1, gi)) { sum += pN; n++; }
    if (n > 0) { out = sum / n; return true; }
  }
  (void)self;
  return false;
}

// ---------------------------------------------- Poisson, wave march -----
//
// One red-black SOR iteration per launch with no LDS and no barriers: every
// wave is an independent tile of 128 columns (2 per lane, 16-byte loads and
// stores) marching down a band of rows, and row neighbours across lanes move
// by DPP wave shifts. 4 columns each side are halo (recomputed), so a wave
// writes 120 columns. At front row R one step loads p_in(R), f(R-1); updates
// red at R-1, black at R-2; refreshes ghosts / solids at R-3; computes the
// residual and stores at R-4. Rows R+1..R+4 of p_in and f are in flight.

// Residual magnitude for the march kernels: as residual_at, but the cavity's
// 0/1 indicator products are selects. Only |r| is used (max-norm), and
// 0*x == +-0 adds nothing to a sum with a non-zero term, so |r| is identical.
template <int CASE>
__device__ __forceinline__ double residual_abs(const Coef& c, int nx, int ny, int j, int i, double pc, double pW,
                                               double pE, double pS, double pN, double fc) {
  if (CASE == CAVITY) {
    const double tE = (i < nx) ? (pE - pc) : 0.0;
    const double tW = (i > 1) ? (pW - pc) : 0.0;
    const double tN = (j < ny) ? (pN - pc) : 0.0;
    const double tS = pS - pc;
    return fabs(c.idx2 * (tE + tW + tN + tS) - fc);
  } else {
    return fabs(residual_at<CASE>(c, nx, ny, j, i, pc, pW, pE, pS, pN, fc));
  }
}

// Convergence test of the residual recorded for iteration kk (launch-start
// test of the reference's while condition, cavity-01.cpp:633): true = go on.
// proof: the slot holds the proof ratio of iteration kk (go on iff > 1)
__device__ __forceinline__ bool pair_go_on(const PoissonCtl& ctl, int kk, int lane, double tol, bool proof = false) {
  double prev;
  if (kk == 0) {
    prev = ctl.tol[1];
  } else {
    const double* slot = ctl.ring + (size_t)(kk & (RING - 1)) * RES_SHARDS * SHARD_STRIDE;
    prev = (lane < RES_SHARDS) ? slot[lane * SHARD_STRIDE] : 0.0;
    prev = wave_max(prev);
    if (proof) return prev > 1.0;
  }
  return prev > tol;
}

// The reference's while condition for the iterations [ka, kb] the host gave
// this launch (the previous launch's, or with the lagged test the one before;
// 0 = the initial residual; others only on check_every multiples): the first
// one that meets the tolerance ends the solve there. Returns false if this
// launch has nothing to do (stopped now or earlier). All waves agree.
// proof (the tested launch ran in proof mode): an iteration the proof does not
// settle ends the proof-mode launches there (stop code 2); the host evaluates
// it exactly.
__device__ __forceinline__ bool window_go_on(const PoissonCtl& ctl, int ka, int kb, int lane, bool first_wave,
                                             bool proof = false) {
  if (ctl.stop[0] != 0) return false;
  const double tol = ctl.tol[0];
  for (int kk = ka; kk <= kb; ++kk) {
    if (!(kk == 0 || (kk >= 1 && kk % ctl.check_every == 0))) continue;
    if (!pair_go_on(ctl, kk, lane, tol, proof)) {
      if (first_wave && lane == 0) {
        ctl.stop[1] = kk;
        ctl.stop[0] = (proof && kk > 0) ? 2 : 1;
      }
      return false;
    }
  }
  return true;
}

// Interior SOR update / residual magnitude: every neighbour is a fluid cell
// (cavity: all four indicators are 1, so the reference's products are the
// plain values). Same operations in the same order as sor_update /
// residual_abs, hence the same bits; no selects.
template <int CASE>
__device__ __forceinline__ double sor_interior(const Coef& c, double pc, double pW, double pE, double pS, double pN,
                                               double fc) {
  if (CASE == CAVITY) return pc * c.one_m_omega + c.om_nc[4] * ((pE + pW) + (pN + pS) - fc * c.h2);
  const double sum = c.idx2 * (pE + pW) + c.idy2 * (pN + pS);
  const double gs = div_denom(c, sum - fc);  // (sum - fc) / denom
  return c.one_m_omega * pc + c.omega * gs;
}
template <int CASE>
__device__ __forceinline__ double residual_interior(const Coef& c, double pc, double pW, double pE, double pS,
                                                    double pN, double fc) {
  if (CASE == CAVITY) return fabs(c.idx2 * ((pE - pc) + (pW - pc) + (pN - pc) + (pS - pc)) - fc);
  const double lap = (pE - 2.0 * pc + pW) * c.idx2 + (pN - 2.0 * pc + pS) * c.idy2;
  return fabs(lap - fc);
}

// SOR update of a boundary-column wave's cell: sor_update<CAVITY> with the
// indicators as lane constants (same operands, same order, same bits)
__device__ __forceinline__ double cav_edge_sor(const Coef& c, bool top, double ce, double cw, double om, double omt,
                                               double pc, double pW, double pE, double pS, double pN, double fc) {
  const double tN = top ? pN * 0.0 : pN;  // row-uniform
  return pc * c.one_m_omega + (top ? omt : om) * ((pE * ce + pW * cw) + (tN + pS) - fc * c.h2);
}

// |residual| of a boundary-column wave's cell (residual_abs<CAVITY> with the
// indicator products; +-0 terms leave |r| unchanged)
__device__ __forceinline__ double cav_edge_res(const Coef& c, bool top, double ce, double cw, double pc, double pW,
                                               double pE, double pS, double pN, double fc) {
  const double tN = top ? (pN - pc) * 0.0 : (pN - pc);
  return fabs(c.idx2 * ((pE - pc) * ce + (pW - pc) * cw + tN + (pS - pc)) - fc);
}

// Proof-mode ratio of one sweep (march.hpp proof_ratio is
// the cavity march's form of the same bound; tile.hip and open.hip use this one). A black cell with four
// neighbours that the sweep's refresh leaves alone has residual
//   r = K (p' - p) + E,   K = d (1 - w) / w,
// d = 4 idx2 (cavity: p' = (1-w) p + (w/4)(S - h^2 f), r = idx2 (S - 4 p') - f)
// or d = 2 (idx2 + idy2) (open cases: p' = (1-w) p + w (S - f) / d,
// r = S - d p' - f, S = idx2 (pE + pW) + idy2 (pN + pS)). The rounding of the
// update (five operations and the correctly rounded divide) and of the
// reference's own evaluation of r stays below 64 u (d P + F) (u = 2^-53, P a
// bound on every |p| the cell's stencils see, F on |f|); the margin used is
// 2^-43 (pm P + F) with pm = idx2 (cavity: the march's constant, 8x its bound)
// or d (16x). A sweep maps P + fd F to at most 9 (P + fd F) (red: |p'| <= 3P
// + 2 fd F, black from those), fd = h^2 (cavity) or 1/d: P <= 9^nsw (Pin + fd F).
// |p' - p| > thr = (tol + margin) / |K| (x (1 + 2^-38)) then proves that the
// reference's computed |r| > tol: its loop goes on. Returns max|p' - p| / thr.
__device__ __forceinline__ double proof_ratio_gen(const Coef& c, double tol, double dmax, double pin, double fmx,
                                                   double growth) {
  const double P = growth * (pin + c.proof_fd * fmx) * (1.0 + 0x1p-40);
  const double margin = 0x1p-43 * (c.proof_pm * P + fmx);
  const double thr = (tol + margin) / c.proof_k * (1.0 + 0x1p-38);
  const double q = dmax / thr;
  return (q == q && q >= 0.0) ? q : 0.0;  // non-finite bounds prove nothing
}


// The SOR launches' p_out rows. CFD_WT_STORE 1: written through (sc1 buffer
// stores): no dirty lines stay in the XCD's L2 at the kernel's end, which the
// next dependent launch would otherwise wait for (MI355X_MICROARCH.md,
// "boundary": + bytes / 6 TB/s). 0: streamed (nt) stores, kept in L2.
#ifndef CFD_WT_STORE
#define CFD_WT_STORE 0
#endif
__device__ __forceinline__ __amdgpu_buffer_rsrc_t out_rsrc(double* base, const Geo& g) {
  // num_records is 32 bits: a buffer past 4 GiB is clamped (the host refuses
  // the CFD_WT_STORE build for such grids: Solver::validate)
  const size_t bytes = (size_t)g.nrows * (size_t)g.pitch * sizeof(double);
  return __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)(unsigned)(bytes < 0xFFFFFFFFull ? bytes : 0xFFFFFFFFull),
                                           0x00020000);
}
__device__ __forceinline__ void store_row_pair(double* base, __amdgpu_buffer_rsrc_t r, size_t off, double2 v) {
#if CFD_WT_STORE
  typedef int v4i __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), r, (int)(off * sizeof(double)), 0, 16);
  (void)base;
#else
  typedef double d2v __attribute__((ext_vector_type(2)));
  d2v mv = {v.x, v.y};
  __builtin_nontemporal_store(mv, reinterpret_cast<d2v*>(base + off));
  (void)r;
#endif
}

// Whether march step GST (0..19: the first two groups of a wave's march; -1:
// a later step) runs an update whose rows enter the band's dependency cone at
// step T + p (p: the march's parity alignment step, 0 or 1): compile-time
// except at step T itself (march.hpp cav_sweeps, lexw.hpp lx_sweeps).
template <int GST, int T>
__device__ __forceinline__ bool cone_step(int p) {
  if constexpr (GST < 0 || GST > T) return true;
  else if constexpr (GST < T) return false;
  else return p == 0;
}

}  // namespace cfd
