// resident.hip — the register-resident SOR solve (resident.hpp has the
// design): red-black with the proof-mode stop rule, and the reference's own
// order with sampled exceedance bits. Own translation unit: device.hpp only.
#include <algorithm>
#include <mutex>
#include <set>
#include <string>
#include <type_traits>
#include <utility>

#include "internal.hpp"
#include "resident.hpp"

namespace cfd {

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
constexpr unsigned long long RES_SPIN_TICKS = 200000000ull;  // 2 s of the 100 MHz wall clock: a wait that long is a bug

// write-through (sc1) 16-B load / store of a column pair (MI355X_MICROARCH.md
// "Valid forms", first row: every store of a handed-off byte sc1 and drained
// before the flag, every load of it sc1)
__device__ __forceinline__ double2 ld_sc1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16));
}
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t r, unsigned off, double2 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), r, (int)off, 0, 16);
}
__device__ __forceinline__ unsigned ld_flag(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Lane constants of the two columns a lane holds (slot a: gx, slot b: gx + 1)
struct ResLane {
  double om_a, om_b;    // omega / nc of the column below the top row (nc = 4 - walls among W, E), 0 at
                        // ghost / outside columns
  double omt_a, omt_b;  // the same in the top row (its north neighbour is the lid's ghost: nc one less)
  double omm_a, omm_b;  // 1 - omega; 1 at ghost / outside columns
  double pa, pb;        // 1.0: a proving cell (owned, 1 < i < nx) of a wave whose rows all prove, else 0.0
  // channel: slot a is the left ghost column (copy E, window two half-sweeps
  // late: ush = 2), slot a / b the right ghost column (0)
  bool lg_a, rg_a, rg_b;
  int ush_a;
  // (tile-uniform) the tile holds the left / right ghost column; the right one
  // sits in slot a (nx + 1 even)
  bool has_lg, has_rg, rg_in_a;
};

// sor_update<CAVITY> (cavity-01.cpp:643-654) as pc * omm + om * sum in every
// cell. The solve's field starts at zero with +0.0 ghosts that never change,
// so a wall's indicator product 0 * p_ghost is +0.0 = p_ghost itself and only
// omega / nc differs at the walls (lexw.hpp lx_upd: the same argument); these
// are per-lane constants, so every wave runs one straight-line update. A
// ghost / outside column takes om = 0, omm = 1: pc * 1 + 0 * sum = pc for
// finite sum and pc != -0.0 (the ghosts are +0.0). Region edge lanes 0 / 63
// and region rows past the halo are updated from zeros: halo, stale anyway
// (they never reach an owned cell within a group; their SOR stays bounded).
// f * h^2 is precomputed (the same rounding).
//
// One half-sweep of colour COL over a wave's RPW rows, in place (a cell's
// neighbours are the other colour). Region row parity = q parity (the plan
// keeps region row 0 on an even grid row), so slot a has colour q & 1. Staged
// over the rows: every stage is independent across rows (RPW chains in
// flight). GEN: a wave holding a ghost row (0, ny + 1), the top row (ny) or
// rows outside the grid - per-row fix-ups (fzm: frozen rows keep their value;
// tpm: the top row's omega / nc), no proofs. Plain waves (every row in 1 ..
// ny - 1) record max |p' - p| of their proving black cells (lane multipliers).
// The reference's order (LEX): cell (j, i) performs its k-th update in
// half-sweep H = i + j + 2(k - 1) (lexw.hpp has the derivation), so a
// half-sweep updates one colour, like red-black, among the cells whose window
// i + j <= H <= i + j + 2(K - 1) holds it (MASK: per-cell selects; groups
// wholly inside every window run unmasked, groups outside all of them skip).
// Its stop rule needs, per iteration, whether some cell's residual exceeds
// tol: one sampled row per wave (RES_QS, owned interior cells) evaluates the
// residual of the other colour's cells in the half-sweep after their update -
// W, S before and E, N after this half-sweep's update, exactly the reference's
// operands (residual_interior<CAVITY>) - and records an exceedance.
#ifndef CFD_RES_QS
#define CFD_RES_QS 3
#endif
constexpr int RES_QS = CFD_RES_QS;  // the sampled row of a wave (odd: a sweep's two samples share one iteration)
#ifndef CFD_RES_OPEN_PROOF_ALL
#define CFD_RES_OPEN_PROOF_ALL 0
#endif
struct LexHalf {
  int u0;          // H - gx - jb: cell (row q, slot a) active iff (unsigned)(u0 - q) <= span; slot b: u0 - q - 1
  unsigned span;   // 2 (K - 1)
  int ks;          // the iteration of this lane's sampled cell in this half-sweep
  unsigned kspan;  // K - 2: sampled iterations 1 .. K - 1 (the cap's is never tested)
  double tol, idx2;
  double2 fs;      // the source of the sampled row
};

template <int RPW, int COL, bool GEN, bool MASK, bool LEX, int Q0, int NQ>
__device__ __forceinline__ void res_half_block(const ResLane& L, double2 (&p)[RPW], const double2* fh,
                                               const double2& Sx, const double2& Nx, unsigned fzm, unsigned tpm,
                                               double& dmx, const LexHalf& lh, bool& ex) {
  double pc[NQ], pw[NQ], pe[NQ], sum[NQ], ns[NQ], nv[NQ];
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    const int q = Q0 + k;
    if ((q & 1) == COL) {
      pc[k] = p[q].x;
      pw[k] = dpp_from_left(p[q].y);
      pe[k] = p[q].y;
    } else {
      pc[k] = p[q].y;
      pw[k] = p[q].x;
      pe[k] = dpp_from_right(p[q].x);
    }
  }
#pragma unroll
  for (int k = 0; k < NQ; ++k) sum[k] = pe[k] + pw[k];
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    const int q = Q0 + k;
    // (the rows below Q0 are already updated in this half-sweep: other colour
    // cells only, the ones read here are unchanged)
    const double2 S = (q == 0) ? Sx : p[q - 1];
    const double2 N = (q == RPW - 1) ? Nx : p[q + 1];
    ns[k] = ((q & 1) == COL) ? (N.x + S.x) : (N.y + S.y);
  }
#pragma unroll
  for (int k = 0; k < NQ; ++k) sum[k] = sum[k] + ns[k];
#pragma unroll
  for (int k = 0; k < NQ; ++k) sum[k] = sum[k] - ((((Q0 + k) & 1) == COL) ? fh[Q0 + k].x : fh[Q0 + k].y);
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    const bool A = ((Q0 + k) & 1) == COL;
    nv[k] = pc[k] * (A ? L.omm_a : L.omm_b) + (A ? L.om_a : L.om_b) * sum[k];
  }
  if constexpr (GEN) {  // (a block without a frozen / top row skips the fix-ups)
    asm volatile("" : "+s"(fzm), "+s"(tpm));
    constexpr unsigned BM = ((1u << NQ) - 1u) << Q0;
    if ((fzm | tpm) & BM) {
#pragma unroll
      for (int k = 0; k < NQ; ++k) {
        const int q = Q0 + k;
        const bool A = (q & 1) == COL;
        if ((tpm >> q) & 1u) nv[k] = pc[k] * (A ? L.omm_a : L.omm_b) + (A ? L.omt_a : L.omt_b) * sum[k];
        if ((fzm >> q) & 1u) nv[k] = pc[k];
      }
    }
  }
  if constexpr (MASK) {  // the reference order's windows (ramps)
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const int q = Q0 + k;
      const unsigned u = (unsigned)(lh.u0 - q - (((q & 1) == COL) ? 0 : 1));
      nv[k] = (u <= lh.span) ? nv[k] : pc[k];
    }
  }
  if constexpr (LEX && !GEN && Q0 <= RES_QS - 1 && Q0 + NQ >= RES_QS + 2) {
    // sampled residual of the other colour's cell c of row RES_QS (iteration
    // lh.ks): W, S before this half-sweep's update, E, N after it
    constexpr int kq = RES_QS - Q0;
    double cv, W, E, fc, mult;
    if constexpr (COL == 1) {  // row RES_QS (odd) updates slot a: c = slot b
      cv = p[RES_QS].y;
      W = pc[kq];
      E = dpp_from_right(nv[kq]);
      fc = lh.fs.y;
      mult = L.pb;
    } else {  // row RES_QS updates slot b: c = slot a
      cv = p[RES_QS].x;
      W = dpp_from_left(pc[kq]);
      E = nv[kq];
      fc = lh.fs.x;
      mult = L.pa;
    }
    const double S = pc[kq - 1], N = nv[kq + 1];  // (rows RES_QS -+ 1 update c's column)
    const double r = fabs(lh.idx2 * ((E - cv) + (W - cv) + (N - cv) + (S - cv)) - fc);
    ex = ex || (r > lh.tol && mult != 0.0 && (unsigned)(lh.ks - 1) <= lh.kspan);
  } else if constexpr (!LEX && !GEN && COL == 1) {
#pragma unroll
    for (int k = 0; k < NQ; ++k) dmx = fmax(dmx, fabs(nv[k] - pc[k]) * ((((Q0 + k) & 1) == COL) ? L.pa : L.pb));
  }
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    if (((Q0 + k) & 1) == COL) p[Q0 + k].x = nv[k];
    else p[Q0 + k].y = nv[k];
  }
}

// the open cases' source in LDS (their p alone fills the registers of 14-row
// waves): planes of slot a / slot b values, [region row][lane] (conflict-free
// 8-B reads; the plane offset fits the reads' immediate offset)
template <int RPW>
__host__ __device__ constexpr int res_fplane() { return RES_MAXW * RPW * 64; }
template <int RPW>
constexpr size_t res_flds_bytes() { return 2 * (size_t)res_fplane<RPW>() * sizeof(double); }

// ---- channel (channel-01.cpp:652-668, 531-541, 672-681) ----
//
// The anisotropic update (sor_update<CHANNEL>: the divide correctly rounded,
// device.hpp div_denom) in every cell, then the ghost rules of the reference's
// refresh after each sweep, as cells of their own colour in the skew
// (lexw.hpp "open cases"): the top ghost row copies its south neighbour and
// the right ghost column is 0, at their own skew time; the bottom ghost row
// copies its north neighbour and the left ghost column its east one, two
// half-sweeps late (the neighbour's previous iteration). Corner ghosts are
// never read: they and the cells outside the grid run the plain update
// (bounded, never stored: the corners' initial values are restored at the
// end). GEN: waves holding a ghost row (per-row fix-ups); EDGE: tiles holding a
// ghost column (per-lane selects).
template <int RPW, int COL, bool GEN, bool EDGE, bool MASK, bool LEX, int Q0, int NQ>
__device__ __forceinline__ void res_half_open(const Coef& c, const ResLane& L, double2 (&p)[RPW], const double* fl,
                                              const double2& Sx, const double2& Nx, unsigned bgm, unsigned tgm,
                                              double& dmx, bool keep, const LexHalf& lh, bool& ex) {
  double pc[NQ], pw[NQ], pe[NQ], pn[NQ], ps[NQ], nv[NQ];
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    const int q = Q0 + k;
    const double2 S = (q == 0) ? Sx : p[q - 1];
    const double2 N = (q == RPW - 1) ? Nx : p[q + 1];
    if ((q & 1) == COL) {
      pc[k] = p[q].x;
      pw[k] = dpp_from_left(p[q].y);
      pe[k] = p[q].y;
      pn[k] = N.x;
      ps[k] = S.x;
    } else {
      pc[k] = p[q].y;
      pw[k] = p[q].x;
      pe[k] = dpp_from_right(p[q].x);
      pn[k] = N.y;
      ps[k] = S.y;
    }
  }
  const double idx2 = c.idx2, idy2 = c.idy2, omm = c.one_m_omega, om = c.omega;
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    const int q = Q0 + k;
    const double fc = fl[((q & 1) == COL ? 0 : res_fplane<RPW>()) + q * 64];
    const double sum = idx2 * (pe[k] + pw[k]) + idy2 * (pn[k] + ps[k]);
    nv[k] = omm * pc[k] + om * div_denom(c, sum - fc);
  }
  // (red-black: the red ghosts keep the stored values in the solve's first
  // half-sweep, `keep` - the reference's first sweep reads them as stored)
  constexpr unsigned BM = ((1u << NQ) - 1u) << Q0;  // this block's rows
  if constexpr (GEN) {  // ghost rows (row-uniform; a block without one skips the selects)
    asm volatile("" : "+s"(bgm), "+s"(tgm));
    if ((bgm | tgm) & BM) {
#pragma unroll
      for (int k = 0; k < NQ; ++k) {
        const int q = Q0 + k;
        if ((bgm >> q) & 1u) nv[k] = keep ? pc[k] : pn[k];
        if ((tgm >> q) & 1u) nv[k] = keep ? pc[k] : ps[k];
      }
    }
  }
  if constexpr (EDGE) {  // ghost columns (lane constants: column 0 is always slot a)
    // (a tile holds at most one of them in most grids, and a row's updated
    // colour holds a ghost cell only in its slot: tile-uniform branches, one
    // select per row where a ghost is updated)
    if (L.has_lg) {
#pragma unroll
      for (int k = 0; k < NQ; ++k)
        if (((Q0 + k) & 1) == COL) nv[k] = L.lg_a ? (keep ? pc[k] : pe[k]) : nv[k];
    }
    if (L.has_rg) {
      if (L.rg_in_a) {
#pragma unroll
        for (int k = 0; k < NQ; ++k)
          if (((Q0 + k) & 1) == COL) nv[k] = L.rg_a ? (keep ? pc[k] : 0.0) : nv[k];
      } else {
#pragma unroll
        for (int k = 0; k < NQ; ++k)
          if (((Q0 + k) & 1) != COL) nv[k] = L.rg_b ? (keep ? pc[k] : 0.0) : nv[k];
      }
    }
  }
  if constexpr (MASK) {  // the skew's windows (the left / bottom ghosts two half-sweeps late)
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const int q = Q0 + k;
      const bool A = (q & 1) == COL;
      int u = lh.u0 - q - (A ? L.ush_a : 1);
      if (GEN && ((bgm >> q) & 1u)) u -= 2;
      nv[k] = ((unsigned)u <= lh.span) ? nv[k] : pc[k];
    }
  }
  if constexpr (LEX && Q0 <= RES_QS - 1 && Q0 + NQ >= RES_QS + 2) {
    // sampled residual (channel-01.cpp:672-681) of the other colour's cell of
    // row RES_QS (2 <= i <= nx-1, 2 <= j <= ny-1: no ghost neighbour)
    constexpr int kq = RES_QS - Q0;
    double cv, W, E, fc, mult;
    if constexpr (COL == 1) {
      cv = p[RES_QS].y;
      W = pc[kq];
      E = dpp_from_right(nv[kq]);
      fc = lh.fs.y;
      mult = L.pb;
    } else {
      cv = p[RES_QS].x;
      W = dpp_from_left(pc[kq]);
      E = nv[kq];
      fc = lh.fs.x;
      mult = L.pa;
    }
    const double S = pc[kq - 1], N = nv[kq + 1];
    const double lap = (E - 2.0 * cv + W) * idx2 + (N - 2.0 * cv + S) * idy2;
    ex = ex || (fabs(lap - fc) > lh.tol && mult != 0.0 && (unsigned)(lh.ks - 1) <= lh.kspan);
  } else if constexpr (!LEX && COL == 1) {
    // red-black proof: max |p' - p| of the proving black cells - of one row
    // per wave (CFD_RES_OPEN_PROOF_ALL 0: any subset of cells proves "the
    // reference goes on" when one of them does; every row's pc kept for it
    // spilled the 14-row kernel), or of every row
#pragma unroll
    for (int k = 0; k < NQ; ++k)
      if (CFD_RES_OPEN_PROOF_ALL || Q0 + k == RES_QS)
        dmx = fmax(dmx, fabs(nv[k] - pc[k]) * ((((Q0 + k) & 1) == COL) ? L.pa : L.pb));
  }
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    if (((Q0 + k) & 1) == COL) p[Q0 + k].x = nv[k];
    else p[Q0 + k].y = nv[k];
  }
}

// rows in scheduling blocks of RES_BLK (16-row waves: bounded live temporaries)
#ifndef CFD_RES_BLK
#define CFD_RES_BLK 8
#endif
#ifndef CFD_RES_BLK_RB
#define CFD_RES_BLK_RB 7
#endif
#ifndef CFD_RES_BLK_OPEN
#define CFD_RES_BLK_OPEN 7
#endif
template <int CASE, int RPW, int COL, bool GEN, bool EDGE, bool MASK, bool LEX, int Q0 = 0>
__device__ __forceinline__ void res_half(const Coef& c, const ResLane& L, double2 (&p)[RPW], const double2* fh,
                                         const double* fl, const double2& Sx, const double2& Nx, unsigned fzm,
                                         unsigned tpm, double& dmx, bool keep, const LexHalf& lh, bool& ex) {
  // (larger waves: smaller blocks; the first block holds the sampled rows RES_QS -+ 1)
  constexpr int BLK = RPW > 8 ? (LEX ? CFD_RES_BLK_OPEN : CFD_RES_BLK_RB) : CFD_RES_BLK;
  static_assert(!LEX || BLK >= RES_QS + 2, "the sampled row and its neighbours in the first block");
  constexpr int NQ = (RPW - Q0) < BLK ? (RPW - Q0) : BLK;
  if constexpr (CASE == CAVITY) res_half_block<RPW, COL, GEN, MASK, LEX, Q0, NQ>(L, p, fh, Sx, Nx, fzm, tpm, dmx, lh, ex);
  else res_half_open<RPW, COL, GEN, EDGE, MASK, LEX, Q0, NQ>(c, L, p, fl, Sx, Nx, fzm, tpm, dmx, keep, lh, ex);
  if constexpr (Q0 + NQ < RPW) {
    __builtin_amdgcn_sched_barrier(0);
    res_half<CASE, RPW, COL, GEN, EDGE, MASK, LEX, Q0 + NQ>(c, L, p, fh, fl, Sx, Nx, fzm, tpm, dmx, keep, lh, ex);
  }
}

// OR across the wave's 64 lanes
__device__ __forceinline__ unsigned long long wave_or64(unsigned long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned lo = (unsigned)v, hi = (unsigned)(v >> 32);
    v |= (unsigned long long)(unsigned)__shfl_xor((int)lo, off, 64) |
         ((unsigned long long)(unsigned)__shfl_xor((int)hi, off, 64) << 32);
  }
  return v;
}
__device__ __forceinline__ unsigned long long ld_bits(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// bounded spin: true = gave up (the wait exceeded RES_SPIN_TICKS)
__device__ __forceinline__ bool res_spin_expired(unsigned long long t0) {
  __builtin_amdgcn_s_sleep(2);
  return wall_clock64() - t0 > RES_SPIN_TICKS;
}

}  // namespace

// diagnostic build only (CFD_RES_STAMPS=1, never the product library): each
// wave sums the shader-clock cycles of its group phases over the solve - 0
// neighbour wait, 1 halo loads, 2 first exchange + proofs, 3 sweeps, 4 group
// end to the drained stores (bands, proofs / bits), 5 the barrier and the
// flag - and counts its groups (6); read back by cfd_res_stamps
// ([tile][wave][7], scripts/dbg/res_stamps.py)
#ifndef CFD_RES_STAMPS
#define CFD_RES_STAMPS 0
#endif
#if CFD_RES_STAMPS
constexpr int RES_STAMP_SEGS = 7;
__device__ unsigned long long res_stamp_buf[256 * RES_MAXW * RES_STAMP_SEGS];
#define RES_STAMP(seg)                                                          \
  do {                                                                          \
    unsigned long long t_;                                                      \
    __builtin_amdgcn_sched_barrier(0);                                          \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                          \
    st_acc[seg] += t_ - st_last;                                                \
    st_last = t_;                                                               \
  } while (0)
#else
#define RES_STAMP(seg) ((void)0)
#endif

// One launch = the whole solve (or, red-black, its replay to a known count:
// RES_REPLAY). LEX: the reference's order.
template <int CASE, int RPW, bool LEX>
__global__ __launch_bounds__(RES_MAXW * 64, 1) void poisson_resident_kernel(Geo g, Coef c, const double* __restrict__ pin,
                                                                             double* __restrict__ pout,
                                                                             const double* __restrict__ f, ResCtl R,
                                                                             ResPlan rp, int flags) {
  constexpr int NS = res_ns(CASE != CAVITY, LEX), H = res_halo(CASE != CAVITY, LEX), TW = res_tw(CASE != CAVITY, LEX);
  __shared__ double2 E[2][RES_MAXW][2][64];  // the waves' first / last rows after each half-sweep (by parity)
  __shared__ double red[2][RES_MAXW][NS + 1];  // red-black: per wave max |p' - p| per sweep, max |p| of the
                                               // input (group parity: wave 0 reads one while the waves write the other)
  __shared__ int dec;                         // 0 go on, 1 exit (fallback / stop), 2 exit (timeout)
  __shared__ int gdec;                        // red-black: the group a fallback starts at; LEX: the open iteration
  extern __shared__ double res_fl[];          // (the open cases) the source, res_fplane planes
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int NW = rp.waves;
  const bool replay = !LEX && (flags & RES_REPLAY) != 0;
  if (threadIdx.x == 0) dec = 0;  // (read after the first barrier)

  // tiles of one XCD next to each other (speed only: blocks b and b + 8 share one)
  const int nblk = (int)gridDim.x;
  const int L8 = (nblk / 8) * 8;
  const int bl = (int)blockIdx.x;
  const int tile = bl < L8 ? (bl % 8) * (nblk / 8) + bl / 8 : bl;
  const int ntiles = rp.ctiles * rp.rtiles;
  const int ct = tile % rp.ctiles, rt = tile / rp.ctiles;
  const int nx = g.nx, ny = g.ny;
  const int x0 = ct * TW, x1 = min(x0 + TW, nx + 2);  // owned columns [x0, x1)
  const int y0 = rp.lo + rt * rp.th, y1 = min(y0 + rp.th, rp.hi);  // owned rows [y0, y1)
  const int gy0 = y0 - H;                    // grid row of region row 0 (even)
  const int RR = (y1 - y0) + 2 * H;          // region rows (<= NW * RPW: host plan)
  const int c0 = x0 - H;                     // grid column of lane 0's slot a
  const int gx = c0 + 2 * lane;              // this lane's columns gx, gx + 1 (gx even)
  const int jb = gy0 + w * RPW;              // grid row of this wave's row 0
  const int rlo = g.row_lo, rhi = g.row_lo + g.nrows - 1;  // stored rows
  const int gxc = min(max(gx, 0), g.pitch - 2);
  const unsigned P = (unsigned)g.pitch;
  // (a row's byte offset from a base made opaque per group: the rows' offsets
  // are recomputed where used instead of hoisted out of the group loop as
  // 2 x RPW live registers - spilled at 14 rows per wave)
  auto offs = [&](int j, unsigned base) { return (unsigned)(j - rlo) * P * 8u + base; };

  // row classes of this wave (wave-uniform): owned rows, halo rows read at each
  // group start; cavity: frozen rows (ghost rows, rows outside the grid), the
  // top row; channel: the bottom (fzm) and top (tpm) ghost rows
  constexpr bool OPEN = CASE != CAVITY;
  unsigned ownm = 0, haloh = 0, fzm = 0, tpm = 0, rowm = 0;
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
    const int r = w * RPW + q, j = jb + q;
    const bool own = j >= y0 && j < y1;
    if (own) ownm |= 1u << q;
    if (r < RR) rowm |= 1u << q;  // region rows (the rest: past the halo, never loaded)
    // region rows read from the neighbours at each group start (grid rows only)
    if (r < RR && !own && j >= 0 && j <= ny + 1) haloh |= 1u << q;
    if (OPEN ? j == 0 : (j <= 0 || j >= ny + 1)) fzm |= 1u << q;
    if (OPEN ? j == ny + 1 : j == ny) tpm |= 1u << q;
  }
  ownm = __builtin_amdgcn_readfirstlane(ownm);
  haloh = __builtin_amdgcn_readfirstlane(haloh);
  fzm = __builtin_amdgcn_readfirstlane(fzm);
  tpm = __builtin_amdgcn_readfirstlane(tpm);
  rowm = __builtin_amdgcn_readfirstlane(rowm);
  const bool gen = (fzm | tpm) != 0u;                       // (wave-uniform) the fix-up path
  // cavity: every row owned and in 1 .. ny - 1 (the proof's cells; the sampled
  // row's cells); channel: the sampled row owned and in 2 .. ny - 1
  // (channel, red-black: every row owned and in 2 .. ny - 1)
  const bool proves = (OPEN && LEX) ? (((ownm >> RES_QS) & 1u) && jb + RES_QS >= 2 && jb + RES_QS <= ny - 1)
                      : OPEN ? (ownm == (1u << RPW) - 1u && jb >= 2 && jb + RPW - 1 <= ny - 1)
                             : (!gen && ownm == (1u << RPW) - 1u);
  // lane constants
  const bool own_pair = gx >= x0 && gx < x1;
  ResLane L;
  {
    const double o2 = c.om_nc[2], o3 = c.om_nc[3], o4 = c.om_nc[4], omw = c.one_m_omega;
    auto col = [&](int i, double& om, double& omt, double& omm, double& pr) {
      const bool in = i >= 1 && i <= nx, wall = i == 1 || i == nx;
      om = !in ? 0.0 : wall ? o3 : o4;
      omt = !in ? 0.0 : wall ? o2 : o3;
      omm = in ? omw : 1.0;
      pr = (proves && own_pair && i >= 2 && i <= nx - 1) ? 1.0 : 0.0;
    };
    col(gx, L.om_a, L.omt_a, L.omm_a, L.pa);
    col(gx + 1, L.om_b, L.omt_b, L.omm_b, L.pb);
    L.lg_a = gx == 0;
    L.rg_a = gx == nx + 1;
    L.rg_b = gx + 1 == nx + 1;
    L.ush_a = gx == 0 ? 2 : 0;
    L.has_lg = c0 <= 0;
    L.has_rg = c0 + 127 >= nx + 1;
    L.rg_in_a = ((nx + 1) & 1) == 0;
  }
  // channel: a tile whose region holds a ghost column (tile-uniform)
  const bool edge = OPEN && (c0 <= 0 || c0 + 127 >= nx + 1);
  const bool col_in = gx >= 0 && gx <= nx + 1;      // a grid column pair (its halo cells are published)
  const bool halo_lane = col_in && !own_pair;       // owned rows: this lane's pair belongs to a neighbour
  const bool band_lane = own_pair && (gx < x0 + H || gx >= x1 - H);  // owned pair in the left / right band

  // the region from p_in (rows / columns clamped to stored memory: clamped
  // cells lie outside the grid, are never updated and never stored), the
  // source as f * h^2 (LEX: the sampled row's source itself too)
  double2 p[RPW], fh[OPEN ? 1 : RPW];
  double* const fl = res_fl + (w * RPW) * 64 + lane;
  LexHalf lh{};
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
    const int jc = min(max(jb + q, rlo), rhi);
    const size_t o = (size_t)(jc - rlo) * (size_t)g.pitch + (size_t)gxc;
    p[q] = *reinterpret_cast<const double2*>(pin + o);
    const double2 F = *reinterpret_cast<const double2*>(f + o);
    if constexpr (OPEN) {
      fl[q * 64] = F.x;
      fl[res_fplane<RPW>() + q * 64] = F.y;
    } else {
      fh[q] = make_double2(F.x * c.h2, F.y * c.h2);
    }
    if (LEX && q == RES_QS) lh.fs = F;
  }
  const double tol = R.tol[0];
  // the reference's loop tests the initial residual first (cavity-01.cpp:633)
  if (!replay && !(R.tol[1] > tol)) {
    if (tile == 0 && threadIdx.x == 0) {
      R.status[0] = 1;
      R.status[1] = 0;
    }
    return;
  }
  const double fmx = R.tol[2];
  const int K = R.K;
  // groups: red-black NS sweeps each; LEX: NS half-sweep pairs of the skewed
  // solve, half-sweeps H = 2 .. nx + ny + 2(K - 1) (cell (ny, nx)'s K-th update)
  // (the open cases: the top ghost's K-th copy one half-sweep after cell (ny, nx))
  const int Hlast = nx + ny + 2 * (K - 1) + (OPEN ? 1 : 0);
  const int G = LEX ? (Hlast - 1 + 2 * NS - 1) / (2 * NS) : res_groups(K);
  lh.span = 2u * (unsigned)(K - 1);
  lh.kspan = (unsigned)(K - 2);
  lh.tol = tol;
  lh.idx2 = c.idx2;
  const int js = jb + RES_QS;  // (LEX) this wave's sampled grid row
  // LEX: the cells of the region that can change (cavity: the grid interior;
  // channel: ghosts too, the left / bottom ones two half-sweeps late): their
  // i + j range
  const int GL = OPEN ? 0 : 1;
  const int smin = max(gy0, GL) + max(c0, GL);
  const int smax = min(gy0 + RR - 1, ny + 1 - GL) + min(c0 + 127, nx + 1 - GL);
  const int lag2 = OPEN ? 2 : 0;
  const __amdgpu_buffer_rsrc_t xr[2] = {
      __builtin_amdgcn_make_buffer_rsrc(R.xa, 0, (int)((unsigned)g.nrows * P * 8u), 0x00020000),
      __builtin_amdgcn_make_buffer_rsrc(R.xb, 0, (int)((unsigned)g.nrows * P * 8u), 0x00020000)};
  // Completion spreads one tile per group: when a tile starts group m, its
  // neighbours have finished group m - 1, theirs m - 2, ..., so every tile has
  // finished group m - DIAM (DIAM: the tile grid's Chebyshev diameter).
  // Red-black: a tile's wave 0 publishes the proofs of group x during group
  // x + 1 (drained before its flag x + 2), so at the start of group m the
  // proofs of every group up to m - DIAM - 1 are published: group
  // m - DIAM - 1 is checked then, with no counter and no grid barrier. LEX:
  // the exceedance bits of group x are drained before the tile's flag x + 1;
  // an iteration k has all its samples once the last cell evaluated it
  // (half-sweep nx + ny + 2k - 1), so at the start of group m every iteration
  // up to kdone(m - DIAM) is checked.
  const int DIAM = max(rp.ctiles, rp.rtiles) - 1;
  auto kdone = [&](int gq) {  // the last iteration whose samples are complete after group gq
    const int a = 2 * NS * (gq + 1) + 2 - nx - ny;
    return a >= 0 ? a / 2 : -((-a + 1) / 2);
  };
  unsigned* const myflag = R.flags + tile;
  // one flag per tile (every wave drained, then a barrier, then wave 0's lane 0
  // stores it); wave 0's lanes 0..7 poll the 3x3 ring's (centre skipped): few
  // pollers, so the polls do not crowd the write-through band stores
  int nflag = -1;
  {
    const int n9 = lane < 4 ? lane : lane + 1;
    const int tr = rt + n9 / 3 - 1, tc = ct + n9 % 3 - 1;
    if (lane < 8 && tr >= 0 && tr < rp.rtiles && tc >= 0 && tc < rp.ctiles) nflag = tr * rp.ctiles + tc;
  }
  auto wait_nb = [&](unsigned e) -> bool {  // false: gave up
    const unsigned long long t0 = wall_clock64();
    for (;;) {
      const bool ok = nflag < 0 || ld_flag(R.flags + nflag) >= e;
      if (__all(ok)) return true;
      if (res_spin_expired(t0)) return false;
    }
  };
  // red-black: proofs of group gq (wave 0): lanes < nsw store "iteration gq*NS + 1 + lane goes on"
  auto publish_proofs = [&](int gq) {
    const int nq = min(NS, K - gq * NS);
    double dm = 0.0, pv = 0.0;
    if (lane < NS + 1)
      for (int v = 0; v < NW; ++v) {
        const double x = red[gq & 1][v][lane];
        if (lane < NS) dm = fmax(dm, x);
        else pv = fmax(pv, x);
      }
    pv = __shfl(pv, NS, 64);
    double growth = 1.0;
    for (int q = 0; q < nq; ++q) growth *= 9.0;
    const double ratio = proof_ratio_gen(c, tol, dm, pv, fmx, growth);
    if (lane < nq && ratio > 1.0)
      __hip_atomic_store(R.proven + gq * NS + 1 + lane, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  // red-black: the reference's while condition for the tested iterations of
  // group gc (every one but the cap, which the loop never tests): lane-wise loads
  auto check_load = [&](int gc) -> bool {
    const int kk = gc * NS + 1 + lane;
    const bool tested = lane < NS && kk <= K - 1 && kk % R.check_every == 0;
    return !tested || ld_flag(R.proven + kk) != 0u;
  };
  // LEX: iterations k0 .. k0 + 7 (<= klast), lane = 8 * (k - k0) + shard:
  // this lane's shard has k's bit (every tested k needs one in some shard)
  auto lex_load = [&](int k0, int klast) -> bool {
    const int k = k0 + (lane >> 3), sh = lane & 7;
    if (k > klast) return true;  // (every iteration, as lexw.hpp / smlex.hip: check_every is the red-black orders')
    const int b = k + R.koff;
    return (ld_bits(R.bits + (size_t)sh * R.bwords + (b >> 6)) >> (b & 63)) & 1ull;
  };
  // the first of k0 .. k0 + 7 (<= klast) with no bit in any shard, or -1
  auto lex_first_open = [&](bool have, int k0, int klast) -> int {
    const unsigned long long m = __ballot(have);
    for (int t = 0; t < 8 && k0 + t <= klast; ++t)
      if (((m >> (8 * t)) & 0xffull) == 0ull) return k0 + t;
    return -1;
  };

#if CFD_RES_STAMPS
  unsigned long long st_acc[RES_STAMP_SEGS] = {}, st_last;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_last)::"memory");
#endif
  int gfail = -1;  // red-black: first group left open (fallback); LEX: the open iteration
  bool pend = true;
  int pend_g = -1;  // (wave 0) red-black: the group whose proofs were loaded at this group's start
  int kc = 0;       // (LEX) iterations 1 .. kc checked
  int pk0 = 0, pk1 = -1;  // (wave 0, LEX) the iterations loaded at this group's start
  for (int gi = 0; gi < G; ++gi) {
    const int nsw = LEX ? NS : min(NS, K - gi * NS);
    const int Hg = 2 + 2 * NS * gi;  // (LEX) the group's first half-sweep
    // ---- group start: the neighbours' edge bands of group gi - 1 (wave 0 waits, the others after a barrier)
    if (gi > 0) {
      if (w == 0 && !wait_nb((unsigned)gi) && lane == 0) dec = 2;
      RES_STAMP(0);
      __syncthreads();
      if (dec == 2) {  // a wait gave up: report, leave p_out alone
        if (threadIdx.x == 0) __hip_atomic_store(R.status + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (the loads stay after the poll)
      const __amdgpu_buffer_rsrc_t xp = xr[(gi - 1) & 1];
      unsigned ob = (unsigned)gxc * 8u;
      asm volatile("" : "+v"(ob));
#pragma unroll
      for (int q = 0; q < RPW; ++q) {
        const bool hrow = (haloh >> q) & 1u;
        const bool orow = (ownm >> q) & 1u;
        if ((hrow && col_in) || (orow && halo_lane)) p[q] = ld_sc1(xp, offs(jb + q, ob));
      }
    }
    pend_g = -1;
    if constexpr (LEX) {  // the iterations every tile has finished sampling (evaluated at this group's end)
      pk1 = -1;
      const int kd = min(K - 1, kdone(gi - DIAM));
      if (w == 0 && gi - DIAM >= 0 && kd > kc) {
        pk0 = kc + 1;
        pk1 = min(kd, kc + 8);
        pend = lex_load(pk0, pk1);
      }
    } else if (w == 0 && !replay && gi - DIAM - 1 >= 0) {  // evaluated at this group's end
      pend_g = gi - DIAM - 1;
      pend = check_load(pend_g);
    }
    // max |p| over the region: the proof's P of this group's sweeps (red-black)
    double pm = 0.0;
    if constexpr (!LEX) {
#pragma unroll
      for (int q = 0; q < RPW; ++q)
        if ((rowm >> q) & 1u) pm = fmax(pm, fmax(fabs(p[q].x), fabs(p[q].y)));
    }
#if CFD_RES_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the halo loads' latency in phase 1)
#endif
    RES_STAMP(1);
    // ---- NS sweeps (red, black), the waves' edge rows through LDS after each half-sweep
    double2 Sx = make_double2(0.0, 0.0), Nx = Sx;
    double dmx[NS];
    unsigned long long exm = 0ull;  // (LEX) bit s: a sampled residual of sweep s exceeds tol
    int par = 0;
    auto exchange = [&]() {
      E[par][w][0][lane] = p[0];
      E[par][w][1][lane] = p[RPW - 1];
      __syncthreads();
      if (w > 0) Sx = E[par][w - 1][1][lane];
      if (w < NW - 1) Nx = E[par][w + 1][0][lane];
      par ^= 1;
    };
    // LEX: the group's activity class (tile-uniform): 0 no cell active in any
    // of its half-sweeps, 1 some (masked), 2 every cell in every one
    int act = 2;
    if constexpr (LEX) {
      const int He = Hg + 2 * NS - 1;
      act = (He < smin || Hg - smax > (int)lh.span + lag2) ? 0
            : (Hg - smax >= lag2 && He - smin <= (int)lh.span) ? 2 : 1;
    }
    if (act != 0) exchange();
    RES_STAMP(2);
    auto sweeps = [&](auto gen_c, auto mask_c) {
      constexpr bool GEN = decltype(gen_c)::value;  // (channel: ghost rows or ghost columns)
      constexpr bool MASK = decltype(mask_c)::value;
      if constexpr (OPEN && !LEX && !MASK) {
        // (the channel's red-black full groups, unrolled: interior waves run the
        // lean update, the ghost waves / tiles the fix-ups)
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          dmx[s] = 0.0;
          bool ex = false;
          res_half<CASE, RPW, 0, GEN, GEN, false, LEX>(c, L, p, fh, fl, Sx, Nx, fzm, tpm, dmx[s], GEN && gi == 0 && s == 0,
                                                       lh, ex);
          exchange();
          res_half<CASE, RPW, 1, GEN, GEN, false, LEX>(c, L, p, fh, fl, Sx, Nx, fzm, tpm, dmx[s], false, lh, ex);
          if (s + 1 < NS) exchange();
        }
        return;
      } else if constexpr (OPEN && !LEX) {
        // (MASK here: the short last group, as a loop in the general variant -
        // its conditional sweeps, unrolled, need ~160 more registers at 14 rows)
        double dv[NS];
#pragma unroll
        for (int t = 0; t < NS; ++t) dv[t] = 0.0;
        bool ex = false;
#pragma unroll 1
        for (int s = 0; s < nsw; ++s) {
          double dm = 0.0;
          res_half<CASE, RPW, 0, true, true, false, LEX>(c, L, p, fh, fl, Sx, Nx, fzm, tpm, dm, gi == 0 && s == 0, lh, ex);
          exchange();
          res_half<CASE, RPW, 1, true, true, false, LEX>(c, L, p, fh, fl, Sx, Nx, fzm, tpm, dm, false, lh, ex);
          if (s + 1 < nsw) exchange();
#pragma unroll
          for (int t = 0; t < NS; ++t) dv[t] = s == t ? dm : dv[t];
        }
#pragma unroll
        for (int t = 0; t < NS; ++t) dmx[t] = dv[t];
        return;
      }
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        dmx[s] = 0.0;
        if (s < nsw) {
          bool ex = false;
          if constexpr (LEX) {
            lh.u0 = Hg + 2 * s - gx - jb;
            lh.ks = (Hg + 2 * s - 1 - gx - js) / 2 + 1;
          }
          res_half<CASE, RPW, 0, GEN, GEN, MASK, LEX>(c, L, p, fh, fl, Sx, Nx, fzm, tpm, dmx[s], !LEX && gi == 0 && s == 0,
                                                      lh, ex);
          exchange();
          if constexpr (LEX) lh.u0 += 1;
          res_half<CASE, RPW, 1, GEN, GEN, MASK, LEX>(c, L, p, fh, fl, Sx, Nx, fzm, tpm, dmx[s], false, lh, ex);
          if (s + 1 < nsw) exchange();
          if constexpr (LEX) exm |= ex ? (1ull << s) : 0ull;
        }
      }
    };
    const bool genw = gen || edge;  // (channel: ghost rows in the wave or ghost columns in the tile)
    if (LEX && act == 1) {
      if (genw) sweeps(std::true_type{}, std::true_type{});
      else sweeps(std::false_type{}, std::true_type{});
    } else if (OPEN && !LEX) {
      if (nsw < NS) sweeps(std::true_type{}, std::true_type{});  // (the short last group: the general loop)
      else if (genw) sweeps(std::true_type{}, std::false_type{});
      else sweeps(std::false_type{}, std::false_type{});
    } else if (act != 0) {
      if (genw) sweeps(std::true_type{}, std::false_type{});
      else sweeps(std::false_type{}, std::false_type{});
    }
    RES_STAMP(3);
    // ---- group end: this wave's proof values / exceedance bits, its part of the edge bands, its flag
    if constexpr (LEX) {
      // lane l's bit s <-> iteration kw - l + s (kw: lane 0's sampled iteration
      // at sweep 0): shift by 63 - l into a 128-bit run, OR the lanes
      const int kw = (Hg - 1 - c0 - js) / 2 + 1;
      const int sh = 63 - lane;
      const unsigned long long lo = exm << sh, hi = sh ? (exm >> (64 - sh)) : 0ull;
      const unsigned long long b0 = wave_or64(lo), b1 = wave_or64(hi);
      if (lane == 0 && (b0 | b1) != 0ull) {
        unsigned long long* Bs = R.bits + (size_t)(tile & 7) * R.bwords;
        const int q0 = kw - 63 + R.koff;  // (>= 0: koff covers the earliest cells)
        const int wd = q0 >> 6, o = q0 & 63;
        if (b0) {
          atomicOr(Bs + wd, b0 << o);
          if (o) atomicOr(Bs + wd + 1, b0 >> (64 - o));
        }
        if (b1) {
          atomicOr(Bs + wd + 1, b1 << o);
          if (o) atomicOr(Bs + wd + 2, b1 >> (64 - o));
        }
      }
    } else if (!replay) {
#pragma unroll
      for (int s = 0; s < NS; ++s) dmx[s] = wave_max(dmx[s]);
      pm = wave_max(pm);
      if (lane == 0) {
#pragma unroll
        for (int s = 0; s < NS; ++s) red[gi & 1][w][s] = dmx[s];
        red[gi & 1][w][NS] = pm;
      }
    }
    {
      const __amdgpu_buffer_rsrc_t xo = xr[gi & 1];
      unsigned ob = (unsigned)gxc * 8u;
      asm volatile("" : "+v"(ob));
#pragma unroll
      for (int q = 0; q < RPW; ++q) {
        const int j = jb + q;
        const bool orow = (ownm >> q) & 1u;
        const bool brow = j < y0 + H || j >= y1 - H;  // (row-uniform) in the bottom / top band
        if (orow && own_pair && (brow || band_lane)) st_sc1(xo, offs(j, ob), p[q]);
      }
    }
    // (red-black) the proofs of group gi - 1, published at this group's end, off
    // the sweeps' register peak; drained before flag gi + 1 like the bands
    if (w == 0 && !replay && !LEX && gi > 0) publish_proofs(gi - 1);
    if constexpr (LEX) {
      if (w == 0 && pk1 >= pk0) {
        const int ko = lex_first_open(pend, pk0, pk1);
        if (ko >= 0 && lane == 0) {  // iteration ko: no sampled cell exceeds tol (left open)
          gdec = ko;
          dec = 1;
        }
        kc = pk1;
      }
    } else if (pend_g >= 0 && !__all(pend) && lane == 0) {  // (wave 0) group pend_g left an iteration open
      gdec = pend_g;
      dec = 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the bands (and wave 0's proofs / bits) drained before the flag
    RES_STAMP(4);
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(myflag, (unsigned)(gi + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    RES_STAMP(5);
#if CFD_RES_STAMPS
    st_acc[6] += 1;
#endif
    if (dec == 1) {  // (every tile decides this at the same group)
      gfail = gdec;
      break;
    }
  }
#if CFD_RES_STAMPS
  if (lane < RES_STAMP_SEGS && tile < 256) {
    unsigned long long v = 0;
#pragma unroll
    for (int q = 0; q < RES_STAMP_SEGS; ++q) v = lane == q ? st_acc[q] : v;
    res_stamp_buf[((size_t)tile * RES_MAXW + w) * RES_STAMP_SEGS + lane] = v;
  }
#endif
  if (gfail < 0 && !replay) {
    // what the loop did not check, once every tile has published everything
    // (red-black: wave 0's flag G + 1 after its last proofs; LEX: flag G):
    // red-black groups max(0, G - DIAM - 1) .. G - 1, LEX iterations kc + 1 .. K - 1
    __syncthreads();  // (red[] of the last group)
    if (w == 0) {
      int d = 0;
      unsigned want = (unsigned)G;
      if constexpr (!LEX) {
        publish_proofs(G - 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(myflag, (unsigned)(G + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        want = (unsigned)(G + 1);
      }
      const unsigned long long t0 = wall_clock64();
      for (int t0i = 0; t0i < ntiles && d == 0; t0i += 64) {
        const int t = t0i + lane;
        for (;;) {
          const bool ok = t >= ntiles || ld_flag(R.flags + t) >= want;
          if (__all(ok)) break;
          if (res_spin_expired(t0)) {
            d = 2;
            break;
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if constexpr (LEX) {
        for (int k0 = kc + 1; k0 <= K - 1 && d == 0; k0 += 8) {
          const int ko = lex_first_open(lex_load(k0, K - 1), k0, K - 1);
          if (ko >= 0) {
            d = 1;
            if (lane == 0) gdec = ko;
          }
        }
      } else {
        for (int gc = max(0, G - DIAM - 1); gc < G && d == 0; ++gc)
          if (!__all(check_load(gc))) {
            d = 1;
            if (lane == 0) gdec = gc;
          }
      }
      if (lane == 0) dec = d;
    }
    __syncthreads();
    if (dec == 1) gfail = gdec;
    if (dec == 2) {
      if (threadIdx.x == 0) __hip_atomic_store(R.status + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
  }
  if (gfail >= 0) {  // red-black: the host replays to gfail * NS; LEX: iteration gfail is left open
    if (tile == 0 && threadIdx.x == 0) {
      R.status[0] = 2;
      R.status[1] = LEX ? gfail : gfail * NS;
    }
    return;
  }
  // the final field: owned cells -> p_out (channel: the corner ghosts, which the
  // reference never writes, keep their initial values)
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
    const int j = jb + q;
    if (((ownm >> q) & 1u) && own_pair) {
      double2 v = p[q];
      if (OPEN && (j == 0 || j == ny + 1)) {
        const double2 v0 = *reinterpret_cast<const double2*>(pin + (size_t)(j - rlo) * (size_t)g.pitch + (size_t)gx);
        if (gx == 0 || gx == nx + 1) v.x = v0.x;
        if (gx + 1 == nx + 1) v.y = v0.y;
      }
      *reinterpret_cast<double2*>(pout + (size_t)(j - rlo) * (size_t)g.pitch + (size_t)gx) = v;
    }
  }
  if (!replay && tile == 0 && threadIdx.x == 0) {
    R.status[0] = 0;
    R.status[1] = K;
  }
}

#if CFD_RES_STAMPS
extern "C" int cfd_res_stamps(unsigned long long* out, int n) {
  const int cap = 256 * RES_MAXW * RES_STAMP_SEGS;
  if (n > cap) n = cap;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(res_stamp_buf), (size_t)n * 8) == hipSuccess ? n : -1;
}
#endif

// the channel's ghost refresh (channel-01.cpp:531-541; corners untouched) of
// a resident red-black solve's final field: its red ghosts took their last
// copy one sweep back (resident.hip: ghosts as cells of their own colour)
__global__ void res_refresh_kernel(Geo g, double* __restrict__ p) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int nx = g.nx, ny = g.ny;
  if (t >= 1 && t <= ny && t >= g.row_lo && t < g.row_lo + g.nrows) {
    p[at(g, t, 0)] = p[at(g, t, 1)];
    p[at(g, t, nx + 1)] = 0.0;
  }
  if (t >= 1 && t <= nx) {
    if (g.row_lo <= 0 && g.row_lo + g.nrows > 1) p[at(g, 0, t)] = p[at(g, 1, t)];
    if (g.row_lo <= ny && g.row_lo + g.nrows > ny + 1) p[at(g, ny + 1, t)] = p[at(g, ny, t)];
  }
}
void res_refresh(const Geo& g, double* p, hipStream_t st) {
  const int n = std::max(g.nx, g.ny) + 1;
  res_refresh_kernel<<<(n + 255) / 256, 256, 0, st>>>(g, p);
}

ResPlan res_plan(int nx, int lo, int hi, int max_tiles, bool open, bool lex) {
  const int TW = res_tw(open, lex), HALO = res_halo(open, lex);
  ResPlan rp{};
  rp.lo = lo;
  rp.hi = hi;
  if ((lo & 1) != 0 || hi <= lo) return ResPlan{};
  rp.ctiles = (nx + 2 + TW - 1) / TW;
  const int rows = hi - lo;
  if (rp.ctiles > max_tiles) return ResPlan{};
  const int rt = std::max(1, max_tiles / rp.ctiles);
  rp.th = (rows + rt - 1) / rt;
  rp.th = std::max(HALO, (rp.th + 1) / 2 * 2);  // even (region row parity), at least one halo deep
  rp.rtiles = (rows + rp.th - 1) / rp.th;
  const int rr = rp.th + 2 * HALO;
  // 8 rows per wave; the channel also RES_RPW_OPEN (its source in LDS leaves
  // room: 4096x512's 102-row regions)
  rp.rpw = rr <= 8 * RES_MAXW ? 8
           : (lex && !open && rr <= 10 * RES_MAXW) ? 10  // (the reference order's deeper groups: taller regions)
           : (open && rr <= RES_RPW_OPEN * RES_MAXW) ? RES_RPW_OPEN
                                                     : 0;
  if (rp.rpw == 0) return ResPlan{};  // a tile's region exceeds the register budget
  rp.waves = (rr + rp.rpw - 1) / rp.rpw;
  return rp;
}

namespace {
using ResKernel = void (*)(Geo, Coef, const double*, double*, const double*, ResCtl, ResPlan, int);

// the kernel instance of a (case, order, rows per wave) and its dynamic LDS
// (the channel's source), or nullptr: no instance for that pair
ResKernel res_kernel(int case_id, bool lex, int rpw, size_t* lds) {
  *lds = 0;
  if (case_id == CAVITY && rpw == 8)
    return lex ? poisson_resident_kernel<CAVITY, 8, true> : poisson_resident_kernel<CAVITY, 8, false>;
  if (case_id == CAVITY && rpw == 10 && lex) return poisson_resident_kernel<CAVITY, 10, true>;
  if (case_id == CHANNEL && rpw == 8) {
    *lds = res_flds_bytes<8>();
    return lex ? poisson_resident_kernel<CHANNEL, 8, true> : poisson_resident_kernel<CHANNEL, 8, false>;
  }
  if (case_id == CHANNEL && rpw == RES_RPW_OPEN) {
    *lds = res_flds_bytes<RES_RPW_OPEN>();
    return lex ? poisson_resident_kernel<CHANNEL, RES_RPW_OPEN, true>
               : poisson_resident_kernel<CHANNEL, RES_RPW_OPEN, false>;
  }
  return nullptr;
}

// dynamic LDS past the static 64 KB needs an attribute per kernel instance and
// device, set once each (its result checked)
void res_kernel_attr(ResKernel k, size_t lds) {
  if (lds == 0) return;
  static std::mutex mu;
  static std::set<std::pair<const void*, int>> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) throw Error(CFD_E_DEVICE, "resident solve: hipGetDevice failed");
  std::lock_guard<std::mutex> lk(mu);
  if (done.count({reinterpret_cast<const void*>(k), dev})) return;
  const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds);
  if (e != hipSuccess)
    throw Error(CFD_E_DEVICE, std::string("resident solve: hipFuncSetAttribute: ") + hipGetErrorString(e));
  done.insert({reinterpret_cast<const void*>(k), dev});
}
}  // namespace

int res_coresident_tiles(int case_id, bool lex, const ResPlan& rp, int n_cu) {
  size_t lds = 0;
  const ResKernel k = res_kernel(case_id, lex, rp.rpw, &lds);
  if (!k || rp.waves <= 0) return 0;
  res_kernel_attr(k, lds);
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(k), rp.waves * 64, lds) !=
      hipSuccess)
    return 0;
  return per_cu * n_cu;
}

void res_launch(int case_id, bool lex, const Geo& g, const Coef& c, const double* pin, double* pout, const double* f,
                const ResCtl& R, const ResPlan& rp, int flags, hipStream_t st) {
  const int n = rp.ctiles * rp.rtiles;
  if (n <= 0) throw Error(CFD_E_STATE, "resident solve: empty plan");
  size_t lds = 0;
  const ResKernel k = res_kernel(case_id, lex, rp.rpw, &lds);
  if (!k) throw Error(CFD_E_STATE, "resident solve: no kernel instance for this case / rows per wave");
  res_kernel_attr(k, lds);
  k<<<dim3(n), dim3(rp.waves * 64), lds, st>>>(g, c, pin, pout, f, R, rp, flags);
}

}  // namespace cfd
