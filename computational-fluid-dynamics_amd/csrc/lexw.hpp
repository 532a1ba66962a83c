// lexw.hpp — the reference's lexicographic SOR, bit for bit, at any grid size.
//
// The reference sweeps j = 1..ny, i = 1..nx in order (cavity-01.cpp:635-654):
// cell (j,i) at iteration k reads W, S at iteration k and E, N, itself at k-1.
// With the 5-point stencil this ordering is exactly a red-black half-sweep
// sequence with a time skew: cell (j,i) performs its iteration k at half-sweep
//     H = i + j + 2(k - 1),
// updating from its neighbours' latest values (W, S reached iteration k at
// H-1; E, N reached k-1 at H-1 and move on only at H+1). So the lexicographic
// solve of K iterations is 2K + nx + ny - 2 red-black half-sweeps in which cell
// (j,i) is updated only while i+j <= H <= i+j+2(K-1): a ramp at the start and
// the end, plain red-black in between (scripts/ in DESIGN.md §2 checks the
// identity against the oracle).
//
// The kernel is the cavity's temporal-blocked march (kernels.hpp, cav_march):
// one wave = 128 columns marching up a band of rows, NS sweeps (2NS half-
// sweeps) per launch, red at R-(2S+1), black at R-(2S+2). What differs:
//  * activity masks on tiles that straddle the ramps (FULL tiles need none,
//    tiles with nothing to do are skipped);
//  * the residual of iteration k (cavity-01.cpp:659-677) needs each cell's
//    neighbours at iteration k, i.e. a red cell's black neighbours W, S before
//    and E, N after the black half-sweep that follows it; a black cell's red
//    neighbours before / after the next red half-sweep. The march keeps each
//    sweep's input rows (ring `in`) next to its output rows (ring `w`) and
//    evaluates, at row R-(2S+3): red cells of sweep S and black cells of sweep
//    S-1 (black cells of a launch's last sweep: in the next launch's sweep 0).
//  * iteration numbers vary along the grid (k = (H - i - j)/2 + 1), so a
//    residual is not a per-launch max: each cell contributes to slot k. The
//    loop's test `res > tol` only needs, per k, whether some cell exceeds the
//    tolerance: a wave ballot per row and sweep goes into a per-wave bit window
//    (slots move by one lane every two rows), flushed once per wave into a
//    global per-slot bitset (atomicOr). The reported residual (max-norm of the
//    last iteration) is recomputed from the final field by a separate pass.
#pragma once

#include "kernels.hpp"

namespace cfd {

constexpr int LEXW_SHARDS = 8;  // copies of the exceedance bitset (by block, ~XCD)

struct LexCtl {
  unsigned long long* bits;  // LEXW_SHARDS x words; bit q of the bitset <-> slot kmax - q
  int words;                 // per shard
  int kmax;                  // slot of bit 0
  const double* tol;         // [0] tolerance, [1] initial residual
  int* stop;                 // [0] converged flag, [1] iteration
};

// slot k has a cell whose |residual| exceeds the tolerance (valid once every
// cell has contributed)
__device__ __forceinline__ bool lexw_slot_exceeds(const LexCtl& L, int k) {
  const int q = L.kmax - k;
  unsigned long long w = 0;
#pragma unroll
  for (int s = 0; s < LEXW_SHARDS; ++s) w |= L.bits[(size_t)s * L.words + (q >> 6)];
  return (w >> (q & 63)) & 1ull;
}

// the reference's while condition for the slots [ka, kb] completed since the
// last test (0 = the primed initial residual): false = stop (recorded once)
__device__ __forceinline__ bool lexw_go_on(const LexCtl& L, int ka, int kb, bool first_wave, int lane) {
  if (L.stop[0] != 0) return false;
  const double tol = L.tol[0];
  for (int k = ka; k <= kb; ++k) {
    const bool go = (k == 0) ? (L.tol[1] > tol) : lexw_slot_exceeds(L, k);
    if (!go) {
      if (first_wave && lane == 0) {
        L.stop[1] = k;
        L.stop[0] = 1;
      }
      return false;
    }
  }
  return true;
}

#define LX_SLOT(X) ((((ROT) + 4 - (X)) % 5 + 10) % 5)
#define LX_S10(X) ((((6 * (ROT) + 5 * (PAR)) % 10 + 9 - (X)) % 10 + 20) % 10)

template <int NS>
struct LexRun {
  double2 w[NS][5];   // sweep S: latest values of rows R-2S .. R-2S-4
  double2 in[NS][5];  // sweep S: the same rows as they entered sweep S
  double2 fr[10];     // source rows R-1 .. R-10
  double2 np[5];      // prefetched p_in rows R .. R+4
  double2 nf[5];      // prefetched f rows R-1 .. R+3
  // exceedance bits, wave-uniform: window bit b <-> slot top - b; bits that
  // leave the window (slot top) are appended to hist (bit e: e-th emission)
  unsigned long long win0, win1, hist0, hist1;
  int top, nemit;
};

// Per-wave context beyond WaveCtx: the launch's half-sweeps and the cap.
struct LexCtx {
  int H0;    // first half-sweep of the launch (even: red)
  int K;     // iterations every cell performs (the cap, or the replayed count)
  double tol;
};

// one red-black half-sweep update of row j (ring slot X), colour COLOR
// (0 red, 1 black) at half-sweep H; MASK: per-cell activity and walls
template <int ROT, int JPAR, int COLOR, bool MASK>
__device__ __forceinline__ void lx_update(const WaveCtx<CAVITY>& x, const LexCtx& lc, double2 (&W)[5], int j, int X,
                                          int H, const double2& fc) {
  double2& m = W[LX_SLOT(X)];
  const double2 bh = W[LX_SLOT(X + 1)], ah = W[LX_SLOT(X - 1)];  // rows j-1 (S), j+1 (N)
  if (!(j > x.rmin && j < x.rmax)) return;                         // row-uniform
  if (((JPAR ^ COLOR) & 1) == 0) {  // slot a (even column gi) has this colour
    const double Lb = dpp_from_left(m.y);
    if (MASK) {
      const double nv = sor_update<CAVITY>(x.c, x.g.nx, x.g.ny, j, x.gi, m.x, Lb, m.y, bh.x, ah.x, fc.x);
      const int s = x.gi + j;
      m.x = (x.fl_a(j) && s <= H && H <= s + 2 * (lc.K - 1)) ? nv : m.x;
    } else {
      m.x = sor_fast<CAVITY>(x, j, m.x, Lb, m.y, bh.x, ah.x, fc.x);
    }
  } else {
    const double Ra = dpp_from_right(m.x);
    if (MASK) {
      const double nv = sor_update<CAVITY>(x.c, x.g.nx, x.g.ny, j, x.gi + 1, m.y, m.x, Ra, bh.y, ah.y, fc.y);
      const int s = x.gi + 1 + j;
      m.y = (x.fl_b(j) && s <= H && H <= s + 2 * (lc.K - 1)) ? nv : m.y;
    } else {
      m.y = sor_fast<CAVITY>(x, j, m.y, m.x, Ra, bh.y, ah.y, fc.y);
    }
  }
}

// |cavity residual| (cavity-01.cpp:659-677) of cell (j, i); interior cells
// below the top row need no indicators
template <bool MASK>
__device__ __forceinline__ double lx_res(const WaveCtx<CAVITY>& x, int j, int i, double pc, double pW, double pE,
                                         double pS, double pN, double fc) {
  if (MASK || j == x.g.ny) return residual_abs<CAVITY>(x.c, x.g.nx, x.g.ny, j, i, pc, pW, pE, pS, pN, fc);
  return residual_interior<CAVITY>(x.c, pc, pW, pE, pS, pN, fc);
}

// Residual stage of sweep S at row j = R - (2S+3): red cells of iteration
// H0+2S, black cells of H0+2S-1 (the previous sweep); one ballot each into
// the exceedance window; the last sweep also stores row j.
template <int S, int NS, int ROT, int PAR, bool MASK>
__device__ __forceinline__ void lx_residual(const WaveCtx<CAVITY>& x, const LexCtx& lc, LexRun<NS>& s, int R,
                                            int lane) {
  const int j = R - (2 * S + 3);
  constexpr int JP = PAR ^ 1;  // parity of j
  const double2 m = s.w[S][LX_SLOT(2 * S + 3)];   // row j, after sweep S
  const double2 nN = s.w[S][LX_SLOT(2 * S + 2)];  // row j+1, after sweep S
  const double2 ij = s.in[S][LX_SLOT(2 * S + 3)];  // row j, before sweep S
  const double2 is = s.in[S][LX_SLOT(2 * S + 4)];  // row j-1, before sweep S
  const double2 fc = s.fr[LX_S10(2 * S + 3)];
  if (!(j >= x.y0 && j < x.y1)) return;  // row-uniform
  if (S == NS - 1 && x.out_lane) {
    double2* dst = reinterpret_cast<double2*>(x.pout + (size_t)(j - x.g.row_lo) * (size_t)x.g.pitch + x.gi);
    typedef double d2v __attribute__((ext_vector_type(2)));
    d2v mv = {m.x, m.y};
    __builtin_nontemporal_store(mv, reinterpret_cast<d2v*>(dst));
  }
  if (!(j >= x.g.j0 && j <= x.g.j1)) return;
  const double Lin = dpp_from_left(ij.y);  // lane l-1, column gi-1, before sweep S
  const double Rfi = dpp_from_right(m.x);  // lane l+1, column gi+2, after sweep S
  double rr, rb;                           // |r| of the red and the black cell of this lane
  int ir, ib;
  if (JP == 0) {  // red at gi (slot a), black at gi+1 (slot b)
    ir = x.gi;
    ib = x.gi + 1;
    rr = lx_res<MASK>(x, j, ir, m.x, Lin, m.y, is.x, nN.x, fc.x);
    rb = lx_res<MASK>(x, j, ib, ij.y, ij.x, Rfi, is.y, nN.y, fc.y);
  } else {  // red at gi+1 (slot b), black at gi (slot a)
    ir = x.gi + 1;
    ib = x.gi;
    rr = lx_res<MASK>(x, j, ir, m.y, ij.x, Rfi, is.y, nN.y, fc.y);
    rb = lx_res<MASK>(x, j, ib, ij.x, Lin, m.y, is.x, nN.x, fc.x);
  }
  bool pr = x.out_lane && rr > lc.tol;
  bool pb = x.out_lane && rb > lc.tol;
  if (MASK) {  // interior cells only, and iterations 1..K
    const int H = lc.H0 + 2 * S;
    const int kr = (H - (ir + j)) / 2 + 1, kb = (H - 1 - (ib + j)) / 2 + 1;
    pr = pr && ir >= 1 && ir <= x.g.nx && (H - (ir + j)) >= 0 && kr <= lc.K;
    pb = pb && ib >= 1 && ib <= x.g.nx && (H - 1 - (ib + j)) >= 0 && kb <= lc.K;
  }
  const unsigned long long mr = __ballot(pr), mb = __ballot(pb);
  // window bit of lane 0's red slot: 2NS - 2S; black: +1 on even rows
  constexpr int br = 2 * NS - 2 * S, bb = br + (JP == 0 ? 1 : 0);
  s.win0 |= mr << br;
  s.win1 |= mr >> (64 - br);
  s.win0 |= mb << bb;
  s.win1 |= mb >> (64 - bb);
}

template <int S, int NS, int ROT, int PAR, bool MASK>
__device__ __forceinline__ void lx_sweeps(const WaveCtx<CAVITY>& x, const LexCtx& lc, LexRun<NS>& s, int R, int lane) {
  if constexpr (S < NS) {
    if constexpr (S == 0) s.in[0][LX_SLOT(0)] = s.w[0][LX_SLOT(0)];
    // red at R-(2S+1) (parity PAR^1) in half-sweep H0+2S, black at R-(2S+2) in H0+2S+1
    lx_update<ROT, PAR ^ 1, 0, MASK>(x, lc, s.w[S], R - (2 * S + 1), 2 * S + 1, lc.H0 + 2 * S,
                                     s.fr[LX_S10(2 * S + 1)]);
    lx_update<ROT, PAR, 1, MASK>(x, lc, s.w[S], R - (2 * S + 2), 2 * S + 2, lc.H0 + 2 * S + 1,
                                 s.fr[LX_S10(2 * S + 2)]);
    lx_residual<S, NS, ROT, PAR, MASK>(x, lc, s, R, lane);
    if constexpr (S + 1 < NS) {
      s.w[S + 1][LX_SLOT(2 * S + 2)] = s.w[S][LX_SLOT(2 * S + 2)];
      s.in[S + 1][LX_SLOT(2 * S + 2)] = s.w[S][LX_SLOT(2 * S + 2)];
    }
    lx_sweeps<S + 1, NS, ROT, PAR, MASK>(x, lc, s, R, lane);
  }
}

template <int NS, int ROT, int PAR, bool MASK>  // PAR = parity of R
__device__ __forceinline__ void lx_step(const WaveCtx<CAVITY>& x, const LexCtx& lc, LexRun<NS>& s, int R, int lane) {
  if constexpr (PAR == 0) {
    // residual slots move down by one every two rows: the window's top slot
    // is final for this wave
    const unsigned long long e = s.win0 & 1ull;
    if (s.nemit < 64) s.hist0 |= e << s.nemit;
    else s.hist1 |= e << (s.nemit - 64);
    s.nemit++;
    s.win0 = (s.win0 >> 1) | (s.win1 << 63);
    s.win1 >>= 1;
    s.top--;
  }
  s.w[0][LX_SLOT(0)] = s.np[LX_SLOT(0)];
  s.fr[LX_S10(1)] = s.nf[LX_SLOT(0)];
  if (MASK) {
    s.np[LX_SLOT(-4)] = x.ld(x.pin, R + 4);
    s.nf[LX_SLOT(-4)] = x.ld(x.f, R + 3);
  } else {
    s.np[LX_SLOT(-4)] = x.ld_fast(x.pin, R + 4);
    s.nf[LX_SLOT(-4)] = x.ld_fast(x.f, R + 3);
  }
  lx_sweeps<0, NS, ROT, PAR, MASK>(x, lc, s, R, lane);
}

// OR `len` bits (bits[0..3], 256 max) into shard `sh` of the bitset at bit q0
__device__ __forceinline__ void lexw_flush(const LexCtl& L, int sh, int q0, const unsigned long long (&b)[4], int len) {
  unsigned long long* G = L.bits + (size_t)sh * L.words;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (c * 64 >= len || b[c] == 0) continue;
    const int q = q0 + c * 64;
    const int w = q >> 6, o = q & 63;  // (q0 >= 0: slots <= kmax)
    if (w >= 0 && w < L.words) atomicOr(&G[w], b[c] << o);
    if (o && w + 1 >= 0 && w + 1 < L.words) atomicOr(&G[w + 1], b[c] >> (64 - o));
  }
}

template <int NS, bool MASK>
__device__ __forceinline__ void lx_march(const WaveCtx<CAVITY>& x, const LexCtx& lc, const LexCtl& L, int y0, int y1,
                                         int c0, int lane, int shard) {
  constexpr int H = 2 * NS + 1;
  const int Rb0 = y0 - H;
  const int Rbeg = Rb0 - (Rb0 & 1);  // even first front row: compile-time colours
  const int nsteps = (y1 - y0) + 2 * H + (Rb0 & 1);
  LexRun<NS> s;
  const double2 z = make_double2(0.0, 0.0);
#pragma unroll
  for (int k = 0; k < 5; ++k)
#pragma unroll
    for (int q = 0; q < NS; ++q) s.w[q][k] = s.in[q][k] = z;
#pragma unroll
  for (int k = 0; k < 10; ++k) s.fr[k] = z;
  {
    constexpr int ROT = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      s.np[LX_SLOT(-q)] = MASK ? x.ld(x.pin, Rbeg + q) : x.ld_fast(x.pin, Rbeg + q);
      s.nf[LX_SLOT(-q)] = MASK ? x.ld(x.f, Rbeg + (q - 1)) : x.ld_fast(x.f, Rbeg + (q - 1));
    }
  }
  // slot of lane 0's red cell at sweep 0 in the residual stage of front row R:
  // B(R) = (H0 - c0 - R + 3 - ((R+1)&1))/2 + 1; window top = B + 2NS, taken
  // one row early because even steps shift first
  s.top = (lc.H0 - c0 - (Rbeg - 2) + 3 - ((Rbeg - 1) & 1)) / 2 + 1 + 2 * NS;
  s.win0 = s.win1 = s.hist0 = s.hist1 = 0ull;
  s.nemit = 0;
  const int top0 = s.top;
  int R = Rbeg;
  for (int st = 0; st < nsteps; st += 10, R += 10) {
    lx_step<NS, 0, 0, MASK>(x, lc, s, R, lane);
    lx_step<NS, 1, 1, MASK>(x, lc, s, R + 1, lane);
    lx_step<NS, 2, 0, MASK>(x, lc, s, R + 2, lane);
    lx_step<NS, 3, 1, MASK>(x, lc, s, R + 3, lane);
    lx_step<NS, 4, 0, MASK>(x, lc, s, R + 4, lane);
    lx_step<NS, 0, 1, MASK>(x, lc, s, R + 5, lane);
    lx_step<NS, 1, 0, MASK>(x, lc, s, R + 6, lane);
    lx_step<NS, 2, 1, MASK>(x, lc, s, R + 7, lane);
    lx_step<NS, 3, 0, MASK>(x, lc, s, R + 8, lane);
    lx_step<NS, 4, 1, MASK>(x, lc, s, R + 9, lane);
  }
  // emitted bits (slots top0 - 1 - e: the first emission is the initial top's
  // bit 0... see below), then the window: one descending run of slots
  // position p <-> slot (top0 - 1) - p... the first shift happens at step 0
  // (R even), emitting bit 0 of the empty window for slot top0 - 0; so
  // position p <-> slot top0 - p for p < nemit, and window bit b <-> slot
  // s.top - b = top0 - nemit - b: position nemit + b. One run, slots descending.
  unsigned long long b[4];
  const int n = s.nemit;  // <= 128
  // b = hist (n bits) | window << n
  b[0] = s.hist0;
  b[1] = s.hist1;
  b[2] = 0ull;
  b[3] = 0ull;
  {
    const int w = n >> 6, o = n & 63;
    unsigned long long v0 = s.win0, v1 = s.win1;
    // OR (v1:v0) << n into b
    if (w == 0) {
      b[0] |= v0 << o;
      b[1] |= o ? ((v0 >> (64 - o)) | (v1 << o)) : v1;
      b[2] |= o ? (v1 >> (64 - o)) : 0ull;
    } else if (w == 1) {
      b[1] |= v0 << o;
      b[2] |= o ? ((v0 >> (64 - o)) | (v1 << o)) : v1;
      b[3] |= o ? (v1 >> (64 - o)) : 0ull;
    } else {
      b[2] |= v0 << o;
      b[3] |= o ? ((v0 >> (64 - o)) | (v1 << o)) : v1;
    }
  }
  if (lane == 0) lexw_flush(L, shard, L.kmax - top0, b, n + 128);
}

// One launch of NS lexicographic-order sweeps (half-sweeps H0 .. H0+2NS-1) on
// one strip, tiled as poisson_multi_kernel (PairPlan, interior column tiles
// use the unmasked march when their whole region is active throughout).
template <int NS>
__global__ __launch_bounds__(256, 2) void poisson_lexw_kernel(Geo g, Coef c, const double* __restrict__ pin,
                                                              double* __restrict__ pout, const double* __restrict__ f,
                                                              LexCtl L, int H0, int K, int ka, int kb, PairPlan pl,
                                                              int flags) {
  constexpr int CH = 8;  // column halo (lanes 0-3 and 60-63)
  constexpr int H = 2 * NS + 1;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (!(flags & 4) && !lexw_go_on(L, ka, kb, blockIdx.x == 0 && wv == 0, lane)) return;

  const int nblk = (int)gridDim.x;
  const int L8 = (nblk / 8) * 8;
  const int bl = (int)blockIdx.x;
  const int blk = (bl < L8) ? (bl % 8) * (nblk / 8) + bl / 8 : bl;
  const int tile = blk * 4 + wv;
  const int ne = (pl.ctiles >= 2) ? 2 : 1;
  const int nbe = pl.nbe0 + pl.nbe1, nbi = pl.nb0 + pl.nb1;
  int band, ctile, th, nb0;
  if (tile < ne * nbe) {
    ctile = (tile < nbe) ? 0 : pl.ctiles - 1;
    band = tile % nbe;
    th = pl.the;
    nb0 = pl.nbe0;
  } else {
    const int t = tile - ne * nbe;
    const int nci = pl.ctiles - ne;
    if (t >= nci * nbi) return;
    ctile = 1 + t % nci;
    band = t / nci;
    th = pl.th;
    nb0 = pl.nb0;
  }
  const int c0 = ctile * PAIR_TWC - CH;
  const int gi = c0 + 2 * lane;
  const bool r0 = band < nb0;
  const int y0 = r0 ? pl.lo0 + band * th : pl.lo1 + (band - nb0) * th;
  const int y1 = min(y0 + th, r0 ? pl.hi0 : pl.hi1);
  if (y0 >= y1) return;

  // activity of the marched region (rows y0-H .. y1-1+H, columns c0 .. c0+127,
  // interior cells only) over this launch's half-sweeps
  const int rlo = max(max(y0 - H, 1), g.row_lo), rhi = min(min(y1 - 1 + H, g.ny), g.row_lo + g.nrows - 1);
  const int clo = max(c0, 1), chi = min(c0 + 127, g.nx);
  const int smin = clo + rlo, smax = chi + rhi;
  const int Hend = H0 + 2 * NS - 1;
  const int last = 2 * (K - 1);
  if (smin > Hend) return;                 // not started: both buffers hold the initial field
  if (smax + last < H0 - 2 * NS) return;   // finished two launches ago: both buffers hold the result
  const bool full = smax <= H0 && smin + last >= Hend && clo == c0 && chi == c0 + 127;

  WaveCtx<CAVITY> x{g, c};
  x.pin = pin; x.pout = pout; x.f = f;
  x.gi = gi;
  x.y0 = y0;
  x.y1 = y1;
  x.rmin = max(g.row_lo, 0);
  x.rmax = min(g.row_lo + g.nrows - 1, g.ny + 1);
  x.pair_ok = gi >= 0 && gi + 1 < g.pitch;
  x.out_lane = x.pair_ok && lane >= CH / 2 && lane < 64 - CH / 2;
  x.icol_a = gi >= 1 && gi <= g.nx;
  x.icol_b = gi + 1 >= 1 && gi + 1 <= g.nx;
  x.open_a = x.open_b = true;
  x.gic = min(max(gi, 0), g.pitch - 2);
  LexCtx lc{H0, K, L.tol[0]};
  const int shard = bl & (LEXW_SHARDS - 1);
  if (full) lx_march<NS, false>(x, lc, L, y0, y1, c0, lane, shard);
  else lx_march<NS, true>(x, lc, L, y0, y1, c0, lane, shard);
}

#undef LX_SLOT
#undef LX_S10

// max-norm residual of a cavity field (cavity-01.cpp:659-677) over the owned
// interior cells: the residual the reference reports after its last sweep
__global__ __launch_bounds__(256) void cavity_resmax_kernel(Geo g, Coef c, const double* __restrict__ p,
                                                            const double* __restrict__ f, double* __restrict__ shards) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j = g.j0 + blockIdx.y * 4 + (threadIdx.x >> 6);
  double m = 0.0;
  if (i >= 1 && i <= g.nx && j >= 1 && j <= g.ny && j <= g.j1) {
    const size_t o = at(g, j, i), P = (size_t)g.pitch;
    m = residual_abs<CAVITY>(c, g.nx, g.ny, j, i, p[o], p[o - 1], p[o + 1], p[o - P], p[o + P], f[o]);
  }
  block_max_to_shard<256>(m, shards, (blockIdx.y * gridDim.x + blockIdx.x) % RES_SHARDS);
}

}  // namespace cfd
