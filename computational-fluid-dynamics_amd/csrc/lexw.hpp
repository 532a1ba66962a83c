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
// the end, plain red-black in between (tests/test_gpu_lexw.py checks the
// result bit for bit against the oracle's restatement of the reference loop).
//
// The kernel is a temporal-blocked wave march like the cavity's red-black one
// (kernels.hpp cav_march): one wave = 128 columns (2 per lane, DPP row
// neighbours) marching DOWN a band of rows, NS sweeps (2NS half-sweeps) per
// launch, each sweep's red and black rows a fixed distance behind the front
// row. What differs:
//  * activity: a launch whose every cell is active in every half-sweep it
//    evaluates (the steady phase) runs the plain march; the launches of the
//    two ramps (the first and last (nx+ny)/2NS of a solve) tile only the rows
//    they touch (LexRamp) and mask per cell only in tiles that straddle a ramp
//    front (LX_ACT: three compares per march step, shared by all rows);
//  * residuals: iteration k's residual (cavity-01.cpp:659-677) needs each
//    cell's W, S neighbours before and E, N after the half-sweep that follows
//    it. Marching down, those are exactly the old and new values of the row
//    being updated, so each row update also evaluates the other colour's
//    residual in the same registers (lx_row). A lane's contributions at front
//    row R all belong to iteration Bd(R) - lane;
//  * convergence: the loop's test `res > tol` only needs, per iteration,
//    whether some cell exceeds the tolerance. Each lane keeps one bit per
//    march step (a pinned per-row flag, no max in the loop), the lanes' masks
//    are merged along the diagonals once per wave and OR-ed into a global
//    per-iteration bitset (8 shards), which the next launches test in order.
//    The reported residual (max-norm of the last iteration) is recomputed from
//    the final field (cavity_resmax_kernel); a stop at k < K replays the solve
//    from its initial field with K = k;
//  * straight-line rows: row-uniform conditions (updated row, top row, output
//    row) become scalar coefficients / thresholds, never branches: branches on
//    them split the march loop and serialised its loads (2x slower).
#pragma once

#include "kernels.hpp"

namespace cfd {

constexpr int LEXW_SHARDS = 8;
#ifndef CFD_LEXW_RAMP_EDGE_FULL
#define CFD_LEXW_RAMP_EDGE_FULL 1  // ramp launches: wholly active edge tiles on the unmasked edge march
#endif
#ifndef CFD_LEXW_W2
#define CFD_LEXW_W2 2  // waves per SIMD the steady kernel must fit at NS = 2 (tuned on MI355X)
#endif
#ifndef CFD_LEXW_W3
#define CFD_LEXW_W3 2  // the same at NS = 3
#endif
#define CFD_LEXW_MIN_WAVES(NS) ((NS) <= 2 ? CFD_LEXW_W2 : CFD_LEXW_W3)  // copies of the exceedance bitset (by block, ~XCD)

// Output columns per wave. A value is exact after s half-sweeps on the wave's
// columns [s, 127-s]; the residual evaluated in half-sweep h reads its east
// neighbour's NEW value (column x+1 after h). At 4 sweeps (h up to 8) the last
// output column must therefore be 127-9 = 118: output columns 8..117 (110,
// lanes 4..58; 10-column right halo). Up to 3 sweeps: 8..119 (112, lanes
// 4..59), the red-black kernels' PAIR_TWC. Rows likewise: a strip's stored
// 8-row halo serves up to 3 sweeps (Solver::lexw_ns keeps strips at 3).
// At 5 sweeps (the cavity on one strip) the left halo grows to 10 columns
// (output column 10 reads column 9 after 9 half-sweeps) and the right one to
// 12: output columns 10..115 (106, lanes 5..57).
__host__ __device__ constexpr int lexw_twc(int ns) { return ns >= 5 ? 106 : ns == 4 ? 110 : PAIR_TWC; }
__host__ __device__ constexpr int lexw_ch(int ns) { return ns >= 5 ? 10 : 8; }

// Ramp-launch tiling: bands of `th` rows from row `row0`; band b holds the
// column tiles ca..cb (the ones its rows touch), numbered from first: band[b]
// = first << 16 | ca << 8 | cb. Waves map to tiles band by band, column tiles
// side by side (their shared halo columns are read together from one L2),
// with no empty tiles (a workgroup holds its slot until its last wave ends).
constexpr int LEXW_RAMP_BANDS = 256;
struct LexRamp {
  int nb, th, row0;
  int wsplit;  // 1: the wall column tiles (first, last) march each band as two half bands (two waves)
  // the step: its crossing column tiles xa .. xa + xn - 1 march the bands that
  // reach the block's edge (band rows blo .. blo + th - 1 with blo + th + xreach
  // >= jb) as two half bands too (xn = 0: none)
  int xa, xn, xreach;
  unsigned band[LEXW_RAMP_BANDS];
};

// ramp launch: the column tile and half band (-1: the whole band) of wave o of
// a band whose tiles are ca .. cb (split tiles take two consecutive waves)
__host__ __device__ inline int lexw_ramp_waves(const LexRamp& rp, int ctiles, int b, int ca, int cb, int o,
                                               int* ctile, int* half) {
  int sp[4], n = 0;
  if (rp.wsplit && ca == 0 && cb >= ca) sp[n++] = 0;
  if (rp.xn > 0 && rp.row0 + (b + 1) * rp.th + rp.xreach >= 0)
    for (int c = max(rp.xa, ca); c <= min(rp.xa + rp.xn - 1, cb); ++c)
      if (c != 0 && c != ctiles - 1) sp[n++] = c;
  if (rp.wsplit && cb == ctiles - 1 && cb > 0) sp[n++] = cb;
  int extra = 0;
  for (int q = 0; q < n; ++q) {
    const int at = sp[q] - ca + extra;
    if (o < at) break;
    if (o == at || o == at + 1) {
      *ctile = sp[q];
      *half = o - at;
      return n;
    }
    ++extra;
  }
  *ctile = ca + o - extra;
  *half = -1;
  return n;  // (the split tiles: the band has cb - ca + 1 + n waves)
}

struct LexCtl {
  unsigned long long* bits;  // LEXW_SHARDS x words; bit q of the bitset <-> iteration q - kmax
  int words;                 // per shard
  int kmax;                  // offset: bit of iteration k is k + kmax (>= 0 for every iteration a wave touches)
  const double* tol;         // [0] tolerance, [1] initial residual
  int* stop;                 // [0] 1: the reference stops at iteration [1]; 2: iteration [1] left open
  int kexact;                // iterations >= kexact have every cell's residual evaluated (full
                             // launches); below it the bits come from sampled rows (LX_SAMPLE)
  double* cscr;              // backwards step: the corner's south neighbour's deferred residual
                             // across a launch boundary: {x-part, p_S, iteration} (lxo_row)
};

// slot k has a cell whose |residual| exceeds the tolerance (valid once every
// cell has contributed)
__device__ __forceinline__ bool lexw_slot_exceeds(const LexCtl& L, int k) {
  const int q = L.kmax + k;
  unsigned long long w = 0;
#pragma unroll
  for (int s = 0; s < LEXW_SHARDS; ++s) w |= L.bits[(size_t)s * L.words + (q >> 6)];
  return (w >> (q & 63)) & 1ull;
}

// Ranks (Solver::lexw_reduce_bits): the exceedance bits of iterations ka .. kb
// as 0 / 1 doubles, all-reduced with max (= OR over the ranks: the stop rule
// is "some cell of the whole grid exceeds tol"), then OR-ed back into shard 0,
// so every rank's launches test the same global bits in the same order.
__global__ void lexw_bits_gather_kernel(LexCtl L, int ka, int kb, double* __restrict__ flags) {
  const int k = ka + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (k <= kb) flags[k - ka] = lexw_slot_exceeds(L, k) ? 1.0 : 0.0;
}
__global__ void lexw_bits_scatter_kernel(LexCtl L, int ka, int kb, const double* __restrict__ flags) {
  const int k = ka + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (k > kb || !(flags[k - ka] > 0.0)) return;
  const int q = L.kmax + k;
  atomicOr(L.bits + (q >> 6), 1ull << (q & 63));
}

// the reference's while condition for the slots [ka, kb] completed since the
// last test (0 = the primed initial residual): false = stop (recorded once).
// A slot below kexact holds the sampled rows only: no exceedance there proves
// nothing, the iteration is left open (stop code 2) for the host to evaluate.
__device__ __forceinline__ bool lexw_go_on(const LexCtl& L, int ka, int kb, bool first_wave, int lane) {
  if (L.stop[0] != 0) return false;
  const double tol = L.tol[0];
  for (int k = ka; k <= kb; ++k) {
    const bool go = (k == 0) ? (L.tol[1] > tol) : lexw_slot_exceeds(L, k);
    if (!go) {
      if (first_wave && lane == 0) {
        L.stop[1] = k;
        L.stop[0] = (k == 0 || k >= L.kexact) ? 1 : 2;
      }
      return false;
    }
  }
  return true;
}

#define LX_SLOT(X) ((((ROT) + 4 - (X)) % 5 + 10) % 5)
#define LX_S10(X) ((((6 * (ROT) + 5 * (PAR)) % 10 + 9 - (X)) % 10 + 20) % 10)

// The march goes DOWN (row R - X*d with d = -1: ring position X holds row
// R + X). Sweep S: red at R+2S+1, black at R+2S+2. Marching down, every value
// a residual of the reference's iteration k needs is at hand while a row is
// updated, so no extra state is kept:
//  * red cell c of row jb = R+2S+2 (iteration of half-sweep H0+2S) during
//    black(S) of row jb: its W (black, before black(S)) and E (black, after)
//    are the old and new values of this very update; N = row jb+1 (black(S)
//    done one step earlier); S = row jb-1 (red(S) done, black(S) not yet);
//  * black cell c' of row jr = R+2S+1 (iteration of half-sweep H0+2S-1)
//    during red(S) of row jr: W', E' = the old / new red values; N' = row
//    jr+1 (red(S) done); S' = row jr-1 (sweep S's front row, red(S) not yet).
//    For S = 0 these are the previous launch's last black half-sweep.
// Lane l's contributions at front row R all belong to the same iteration,
// Bd(R) - l with Bd(R) = (H0 - c0 - R - (R&1) - 2)/2 + 1 (sweeps and colours
// alike): at march step t (R = Rbeg - t, Rbeg even) that is Bd0 + t/2 - l. A
// step's residuals are max-reduced in registers, compared with the tolerance
// once, and recorded as bit t/2 of a per-lane mask (VALU only: scalar work in
// the march stalls the wave); the lanes' masks are merged along the
// diagonals (iteration = Bd0 + t/2 - l) once per wave.

// backwards step: the corner's south neighbour's pending residual (lxo_row)
struct LxDefer {
  double xp, ps;
  int k;  // iteration of the pending residual, -1: none
};

template <int NS>
struct LexRun {
  double2 w[NS][5];  // sweep S: rows R+2S .. R+2S+4
  double2 fr[10];    // source rows R+1 .. R+10
  double2 np[5];     // prefetched p_in rows R .. R-4
  double2 nf[5];     // prefetched f rows R+1 .. R-3
  unsigned long long mask;  // bit t/2: a residual of this lane's iteration Bd0 + t/2 - lane exceeds tol
  LxDefer d;         // backwards step: the corner's south neighbour's pending residual (lxo_row)
};

// Per-wave context beyond WaveCtx: the launch's half-sweeps and the cap.
struct LexCtx {
  int H0;    // first half-sweep of the launch (even: red)
  int K;     // iterations every cell performs (the cap, or the replayed count)
  double tol;
  double o2, o3, o4;  // omega / nc (Coef::om_nc) held as values: a select of
                      // Coef fields becomes a select of addresses and a load
  // open cases (lxo_row): the row refreshed as a copy of the row below it,
  // at its own skew time (the top ghost row ny + 1; in the step's column
  // tiles left of its column, the block's bottom row: the rows above it never
  // change), the last row with residuals, and what the copy adds to the value
  // (-0.0: an exact copy, the ghost rule; +0.0: the step's solid refresh
  // 0.0 + p_S, backwards_step-01.cpp:708-738, which turns -0.0 into +0.0)
  int jg, jr1;
  double gz;
};

// Row R of a field at this lane's column pair, row and column clamped to
// stored memory and no select on the value (a select would wait for the load
// and defeat the prefetch): values of rows / lanes outside the grid only feed
// cells that are never updated (ghost rows and columns, halo edges) and are
// never stored.
__device__ __forceinline__ double2 lx_ld(const WaveCtx<CAVITY>& x, const double* base, int R) {
  const int Rc = min(max(R, x.rmin), x.rmax);
  return *reinterpret_cast<const double2*>(base + (size_t)(Rc - x.g.row_lo) * (size_t)x.g.pitch + x.gic);
}

// MODE LX_ACT: per-cell activity masks (tiles on the ramps); 0: every cell
// active in every half-sweep of the launch. Wall columns (the first and last
// column tile, `edge`) take wave-uniform branches inside the same code.
// Cell (j,i) is active in half-sweep H iff i+j <= H <= i+j+2(K-1). Every row
// the march touches at front row R is j = R+X in half-sweep H0+h with h-X =
// -1 (red at X = 2S+1 in H0+2S, black at 2S+2 in H0+2S+1), so with u = H0-1
// -gi-R the update of column gi is active iff 0 <= u <= 2(K-1), of gi+1 iff
// that holds for u-1, and the residual (half-sweep H-1) of gi / gi+1 for u-1
// / u-2: three compares per march step, shared by all 2NS rows.
// (LX_PIN: the masked values are pinned with an empty asm before their
// selects; otherwise the compiler sinks the updates into exec-masked branches,
// which split the march loop into dozens of blocks, serialise its loads and
// ran the ramp launches at half the steady kernel's speed.)
constexpr int LX_ACT = 1;
// 1: the channel's row-checked marches run their groups of 10 steps clear of
// the ghost rows unchecked (lx_march)
#ifndef CFD_LEXW_GROUPS
#define CFD_LEXW_GROUPS 1
#endif
// A/B build only: every interior band of the open cases on the row-checked
// march (one interior code path in the kernel: is the checked path slow for
// its work or for the instruction cache it shares with the safe path?)
#ifndef CFD_LEXW_ALLRC
#define CFD_LEXW_ALLRC 0
#endif
constexpr int LX_SAMPLE = 2;  // sampled residual rows (lx_res_row)
struct LxAct {
  bool a, b, c;    // u, u-1, u-2 within [0, 2(K-1)]
  bool a2, b2;     // u-2, u-3: the same two half-sweeps later (open cases: the left / bottom ghosts)
  unsigned u;      // (the step's corner logic: u == 0 is slot a's first iteration)
};
template <int MODE, bool U = false>
__device__ __forceinline__ LxAct lx_act(const LexCtx& lc, int gi, int R) {
  if constexpr (!(MODE & LX_ACT) && !U) return LxAct{true, true, true, true, true, 0u};
  const unsigned span = 2u * (unsigned)(lc.K - 1);
  unsigned u = (unsigned)(lc.H0 - 1 - R - gi);
  asm volatile("" : "+v"(u));  // (opaque: no loop splitting on the induction variable R)
  if constexpr (!(MODE & LX_ACT)) return LxAct{true, true, true, true, true, u};
  return LxAct{u <= span, u - 1u <= span, u - 2u <= span, u - 2u <= span, u - 3u <= span, u};
}

// SOR update (cavity-01.cpp:643-654) as pc*omm + om*sum in every cell. The
// solve's field starts at zero with +0.0 ghosts that never change, so a wall's
// indicator product 0*p_ghost is +0.0 = p_ghost itself: only omega/nc differs
// at the walls (nc = 4 - walls among W, E, N; es = 1 always). A cell that is
// not updated (ghost rows and columns, rows outside the stored strip) takes om
// = 0, omm = 1: pc*1 + 0*sum = pc for finite sum and pc != -0.0 (the field is
// never -0.0: a sum is -0.0 only when both terms are). Interior tiles choose
// om / omm per row (row-uniform: scalar selects, no vector work); wall tiles
// (EDGE) per lane from values fixed for the wave (LxCol).
struct LxCol {
  int k;  // column kind: 0 outside the grid, 1 wall (i = 1 or nx), 2 interior
};
__device__ __forceinline__ LxCol lx_col(const WaveCtx<CAVITY>& x, int i) {
  const bool in = i >= 1 && i <= x.g.nx;
  const bool wall = (i == 1) || (i == x.g.nx);
  return LxCol{!in ? 0 : wall ? 1 : 2};
}
template <bool EDGE>
__device__ __forceinline__ double lx_upd(const WaveCtx<CAVITY>& x, const LexCtx& lc, bool upd, bool top,
                                         const LxCol& cc, double pc, double pW, double pE, double pS, double pN,
                                         double fc) {
  const double sum = (pE + pW) + (pN + pS) - fc * x.c.h2;
  const double oi = upd ? (top ? lc.o3 : lc.o4) : 0.0;  // row-uniform
  double om, omm;
  if constexpr (EDGE) {  // (a kind per lane, not per-lane coefficients: registers)
    const double ow = upd ? (top ? lc.o2 : lc.o3) : 0.0;
    om = cc.k == 2 ? oi : cc.k == 1 ? ow : 0.0;
    omm = (upd && cc.k != 0) ? x.c.one_m_omega : 1.0;
  } else {
    om = oi;
    omm = upd ? x.c.one_m_omega : 1.0;
  }
  return pc * omm + om * sum;
}

// |residual| (cavity-01.cpp:659-677) in residual_interior's order with the
// north term scaled by eN (0 in the top row, 1 below): (pN-pc)*1 is exact and
// the sign of a zero term cannot change |r|. Wall tiles (EDGE) take
// residual_abs's selects for the east / west terms.
template <bool EDGE>
__device__ __forceinline__ double lx_res(const WaveCtx<CAVITY>& x, double eN, int i, double pc, double pW, double pE,
                                         double pS, double pN, double fc) {
  const double tE = (!EDGE || i < x.g.nx) ? (pE - pc) : 0.0;
  const double tW = (!EDGE || i > 1) ? (pW - pc) : 0.0;
  return fabs(x.c.idx2 * (tE + tW + (pN - pc) * eN + (pS - pc)) - fc);
}

// Update of row j = R + X (colour COLOR) and, from the old and new values, the
// test |residual| > tol of the other colour's cell of this lane (iteration of
// half-sweep H-1; false for rows outside the wave's output rows and, in edge /
// ramp tiles, for cells outside the grid or inactive at H-1). Straight-line
// code: branches on the row-uniform conditions split the march loop and
// serialise its loads, so they become scalar coefficients and thresholds.
template <int ROT, int JPAR, int COLOR, int MODE, bool EDGE, bool STORE, bool RES, bool UP = false>
__device__ __forceinline__ void lx_row(const WaveCtx<CAVITY>& x, const LexCtx& lc, const LxCol (&cc)[2],
                                       double2 (&W)[5], int j, int X, const LxAct& act, const double2& fc, int& exi) {
  double2& m = W[LX_SLOT(X)];
  // rows j+1 (N), j-1 (S): ring position X+1 holds row j+1 marching down, j-1 marching up (lx_march UP)
  const double2 nb = W[LX_SLOT(UP ? X - 1 : X + 1)], sb = W[LX_SLOT(UP ? X + 1 : X - 1)];
  const double2 old = m;
  const bool upd = j > x.rmin && j < x.rmax;  // row-uniform (rows 1..ny: rmin/rmax exclude the ghost rows)
  const bool top = j == x.g.ny;
  // this colour's slot: a (even column gi) iff (j + COLOR) even
  constexpr bool A = ((JPAR ^ COLOR) & 1) == 0;
  if constexpr (A) {
    double nv = lx_upd<EDGE>(x, lc, upd, top, cc[0], m.x, dpp_from_left(m.y), m.y, sb.x, nb.x, fc.x);
    m.x = ((MODE & LX_ACT) && !act.a) ? m.x : nv;
  } else {
    double nv = lx_upd<EDGE>(x, lc, upd, top, cc[1], m.y, m.x, dpp_from_right(m.x), sb.y, nb.y, fc.y);
    m.y = ((MODE & LX_ACT) && !act.b) ? m.y : nv;
  }
  if (STORE && j >= x.y0 && j < x.y1 && x.out_lane) {
    double2* dst = reinterpret_cast<double2*>(x.pout + (size_t)(j - x.g.row_lo) * (size_t)x.g.pitch + x.gi);
    typedef double d2v __attribute__((ext_vector_type(2)));
    d2v mv = {m.x, m.y};
    __builtin_nontemporal_store(mv, reinterpret_cast<d2v*>(dst));
  }
  // residual of the other colour's cell of this lane (iteration of half-sweep
  // H-1), tested against +inf outside the wave's output rows; RES = false:
  // a row the sampled launch does not evaluate (lx_sweeps)
  if constexpr (!RES || UP) return;
  const bool rrow = j >= x.y0 && j < x.y1 && j >= x.g.j0 && j <= x.g.j1;  // row-uniform
  const double thr = rrow ? lc.tol : __builtin_huge_val();
  const double eN = top ? 0.0 : 1.0;
  bool ex;
  if constexpr (A) {  // updated: slot a (gi); the other colour is at gi+1: W = gi (old), E = gi+2 (lane l+1, new)
    ex = lx_res<EDGE>(x, eN, x.gi + 1, m.y, old.x, dpp_from_right(m.x), sb.y, nb.y, fc.y) > thr;
    if constexpr (EDGE) ex = ex && x.icol_b;
    if constexpr ((MODE & LX_ACT) != 0) ex = ex && act.c;
  } else {  // updated: slot b (gi+1); the other colour is at gi: W = gi-1 (lane l-1, old), E = gi+1 (new)
    ex = lx_res<EDGE>(x, eN, x.gi, m.x, dpp_from_left(old.y), m.y, sb.x, nb.x, fc.x) > thr;
    if constexpr (EDGE) ex = ex && x.icol_a;
    if constexpr ((MODE & LX_ACT) != 0) ex = ex && act.b;
  }
  // (an int flag per lane, pinned row by row: a test deferred by the
  // scheduler keeps its residual live, dozens of them across the loop)
  exi = ex ? 1 : exi;
  asm volatile("" : "+v"(exi));
}

// ---- open cases (channel) ----
//
// The reference's anisotropic update (channel-01.cpp:659-666, the divide
// correctly rounded: kernels.hpp div_denom) in every interior cell. Its ghost
// refresh after each sweep (applyPressureGhosts, channel-01.cpp:531-541: p[j][0]
// = p[j][1], p[j][nx+1] = 0, p[0][i] = p[1][i], p[ny+1][i] = p[ny][i], corners
// untouched) fits the skew as cells with a copy rule, updated in the half-sweep
// of their colour:
//  * a ghost AFTER its interior neighbour in the reference's order (top row
//    ny+1, right column nx+1) takes its k-th value at its own skew time
//    i+j+2(k-1), one half-sweep after the neighbour's iteration k: the copy
//    (or 0) the neighbour reads in iteration k+1 as p_prev;
//  * a ghost BEFORE it (left column 0, bottom row 0) is read by the neighbour as
//    p_new, refreshed by the previous sweep, so it copies the neighbour's
//    iteration k-1 value at i+j+2(k-1) for k = 2 .. K+1: two half-sweeps later
//    than a cell of its position (the reference's first sweep reads the stored
//    ghost; the last copy is the refresh after sweep K).
// Residuals (channel-01.cpp:672-681) see the ghosts refreshed after the sweep:
// a top / right ghost is updated in the half-sweep the residual is evaluated
// in (its new value is at hand); a left / bottom one is not yet, so the
// interior cell's own value stands in for it (the copy it will take).
// Interior bands whose march stays off the ghost rows and the halo edges take
// the unmasked update (RC = false); the others choose per row (row-uniform).
struct LxoCol {
  int ka, kb;  // per slot: 0 keep (outside the grid), 1 left ghost, 2 right ghost, 3 interior
  int sa, sb;  // backwards step, per slot: column i < step_i (0), == step_i (1), > step_i (2)
};
__device__ __forceinline__ int lxo_kind(const WaveCtx<CAVITY>& x, int i) {
  return (i < 0 || i > x.g.nx + 1) ? 0 : (i == 0) ? 1 : (i == x.g.nx + 1) ? 2 : 3;
}
__device__ __forceinline__ int lxs_class(const WaveCtx<CAVITY>& x, int i) {
  return (i < x.c.step_i) ? 0 : (i == x.c.step_i) ? 1 : 2;
}

// ---- backwards step (backwards_step-01.cpp:685-740, 872-939) ----
//
// Solid block: i <= si (step_i), j >= jb (inlet_jmax + 1). The reference
// refreshes, after each sweep, the solid cells next to fluid to the mean of
// their fluid neighbours (p_sum starts at 0.0, so one neighbour gives 0.0 + p,
// which turns -0.0 into +0.0). In the skew (requires si >= 2, jb <= ny - 1):
//  * bottom-row solids (jb, i < si): 0.0 + p_S, read by their south neighbour
//    as p_prev: like the top ghost, a copy at their own skew time;
//  * step-column solids (j > jb, si): 0.0 + p_E, read by their east neighbour
//    as p_new: like the left ghost, two half-sweeps later;
//  * the corner (jb, si) = ((0.0 + p_E) + p_S) / 2 with E = (jb, si+1),
//    S = (jb-1, si): S's iteration k+1 and E's iteration k share a half-sweep,
//    and S needs the corner of E(k). The march updates E's row first, so S's
//    update computes the corner from E's new and its own old value, uses it as
//    p_N and writes it into the corner's register, where E's next update and
//    E's residual read it; the corner itself is kept (the final field's corner
//    is refreshed after the solve, Solver::step_corner). S's own residual needs
//    that corner too, one half-sweep after it is evaluated: its x part and p_S
//    wait in registers (or, across a launch boundary, in LexCtl::cscr) until
//    S's next update, which ORs the bit of its iteration directly. Sampled
//    launches skip that one cell.
//  * interior solids never change (both buffers hold them).
// Residuals read the solids refreshed after the sweep: a bottom-row one is
// updated in the residual's half-sweep (new value at hand); a step-column one
// not yet, so the cell's own value stands in (0.0 + p_c).

template <int CASE, bool EDGE, bool RC, bool STEP>
__device__ __forceinline__ double lxo_value(const WaveCtx<CAVITY>& x, int rk, int ck, int rs, int cs, double pc,
                                            double pW, double pE, double pS, double pN, double fc, double gz) {
  const double sor = sor_update<CASE>(x.c, 0, 0, 0, 0, pc, pW, pE, pS, pN, fc);
  if constexpr (!RC && !EDGE) return sor;
  double nv = sor;
  if constexpr (STEP) {  // row class rs: 0 below the block, 1 its bottom row, 2 above (row-uniform)
    const double solid = (rs == 1) ? ((cs == 0) ? 0.0 + pS : pc) : ((cs == 0) ? pc : 0.0 + pE);
    nv = (rs == 0 || cs == 2) ? sor : solid;
  }
  if constexpr (EDGE) nv = (ck == 3) ? nv : (ck == 1) ? pE : (ck == 2) ? 0.0 : pc;
  if constexpr (RC) {  // row kinds: 1 bottom ghost (copy N), 2 top ghost (copy S + gz), 3 keep
    const double g = (rk == 1) ? pN : pS + gz;
    if (EDGE) nv = (rk == 0) ? nv : (rk != 3 && ck == 3) ? g : pc;
    else nv = (rk == 0) ? nv : (rk != 3) ? g : pc;
  }
  return nv;
}

template <int CASE, int ROT, int JPAR, int COLOR, int MODE, bool EDGE, bool RC, bool STORE, bool RES, bool FIRSTH,
          bool LASTH, bool UP = false>
__device__ __forceinline__ void lxo_row(const WaveCtx<CAVITY>& x, const LexCtx& lc, const LexCtl& L, const LxoCol& cc,
                                        double2 (&W)[5], int j, int X, const LxAct& act, const double2& fc, int& exi,
                                        LxDefer& d, double2* nxt = nullptr) {
  // the step's general tiles (block boundary, ghosts): per-cell solid rules
  constexpr bool STEP = CASE == BACKSTEP && EDGE && RC;
  static_assert(!UP || (!EDGE && !RC), "upward march: the open cases' unchecked interior bands");
  constexpr bool FULL = !(MODE & LX_SAMPLE);
  double2& m = W[LX_SLOT(X)];
  double2& mn = W[LX_SLOT(UP ? X - 1 : X + 1)];
  const double2 nb = mn, sb = W[LX_SLOT(UP ? X + 1 : X - 1)];  // rows j+1 (N), j-1 (S)
  const double2 old = m;
  // row kind (row-uniform): 0 interior, 1 bottom ghost, 2 top ghost (or the
  // step's bottom solid row in a left tile: LexCtx::jg), 3 keep (halo edge /
  // outside; the rows above jg)
  const int rk = !RC ? 0 : (j == 0) ? 1 : (j == lc.jg) ? 2 : (j > x.rmin && j < x.rmax) ? 0 : 3;
  const int jb = x.c.inlet_jmax + 1;
  const int rs = !STEP ? 0 : (j < jb) ? 0 : (j == jb) ? 1 : 2;  // (row-uniform)
  const bool rowc = STEP && j == jb - 1 && rk == 0;              // the corner's south neighbour's row
  const int Hh = lc.H0 + X - 1;                                   // this half-sweep
  const int c0k = x.c.step_i + jb - 1;                            // i + j of the corner's south neighbour
  constexpr bool A = ((JPAR ^ COLOR) & 1) == 0;
  if constexpr (A) {
    // the corner's south neighbour (column si in slot a): p_N = the corner of E's new value
    const bool isc = rowc && cc.sa == 1;
    const bool first = act.u == 0u;
    const double cv = ((0.0 + nb.y) + m.x) * 0.5;  // E = (jb, si+1) is slot b of this lane in row jb
    const double pN = (isc && !first) ? cv : nb.x;
    const double nv = lxo_value<CASE, EDGE, RC, STEP>(x, rk, cc.ka, rs, cc.sa, m.x, dpp_from_left(m.y), m.y, sb.x,
                                                      pN, fc.x, lc.gz);
    bool on = true;
    if constexpr ((MODE & LX_ACT) != 0) {
      // left / bottom ghost and step-column solid: two half-sweeps later. (The
      // left ghosts of the block's rows copy solids: the bottom-row one is
      // refreshed after them in the skew like a top ghost, so its ghost keeps
      // the natural time and copies its previous value, as the reference's
      // ghost pass, which runs before the solid pass, does; interior solids are
      // constant either way.)
      const bool lg = EDGE && cc.ka == 1 && !(STEP && rs != 0);
      const bool shifted = (RC && rk == 1) || lg || (STEP && rk == 0 && rs == 2 && cc.sa == 1);
      on = shifted ? act.a2 : act.a;
      m.x = on ? nv : m.x;
    } else {
      m.x = nv;
    }
    if constexpr (STEP) {
      if (isc && on && !first) {  // the corner's register (row jb, column si)
        mn.x = cv;
        // in a black half-sweep row jb has already moved on: to the next
        // sweep's ring (nxt), or, in the last sweep, to p_out
        if (nxt) nxt->x = cv;
        if (STORE && j + 1 >= x.y0 && j + 1 < x.y1 && x.out_lane) x.pout[at(x.g, j + 1, x.gi)] = cv;
      }
      if constexpr (FULL && RES) {  // the pending residual of the previous iteration (deferred)
        const bool own = isc && on && x.out_lane && j >= x.y0 && j < x.y1;
        const int kc = (Hh - c0k) / 2 + 1;  // this update's iteration
        double xp = d.xp, ps = d.ps;
        int kd = d.k;
        if (FIRSTH && own && kd != kc - 1) {  // evaluated in the previous launch's last half-sweep
          xp = L.cscr[0];
          ps = L.cscr[1];
          const double kdd = L.cscr[2];
          kd = (kdd == kdd) ? (int)kdd : -1;  // (NaN: nothing pending)
        }
        if (own && kd == kc - 1 && !first) {
          const double r = xp + ((cv - 2.0 * old.x) + ps) * x.c.idy2 - fc.x;
          if (fabs(r) > lc.tol) {
            const int q = L.kmax + kd;
            atomicOr(&L.bits[q >> 6], 1ull << (q & 63));
          }
        }
        if (isc) d.k = -1;
      }
    }
  } else {  // (column 0 is always slot a)
    const bool isc = rowc && cc.sb == 1;
    const bool first = act.u == 1u;  // slot b: u - 1 == 0
    const double cv = ((0.0 + dpp_from_right(nb.x)) + m.y) * 0.5;  // E = slot a of lane + 1 in row jb
    const double pN = (isc && !first) ? cv : nb.y;
    const double nv = lxo_value<CASE, EDGE, RC, STEP>(x, rk, cc.kb, rs, cc.sb, m.y, m.x, dpp_from_right(m.x), sb.y,
                                                      pN, fc.y, lc.gz);
    bool on = true;
    if constexpr ((MODE & LX_ACT) != 0) {
      const bool shifted = (RC && rk == 1) || (STEP && rk == 0 && rs == 2 && cc.sb == 1);
      on = shifted ? act.b2 : act.b;
      m.y = on ? nv : m.y;
    } else {
      m.y = nv;
    }
    if constexpr (STEP) {
      if (isc && on && !first) {
        mn.y = cv;
        if (nxt) nxt->y = cv;
        if (STORE && j + 1 >= x.y0 && j + 1 < x.y1 && x.out_lane) x.pout[at(x.g, j + 1, x.gi + 1)] = cv;
      }
      if constexpr (FULL && RES) {
        const bool own = isc && on && x.out_lane && j >= x.y0 && j < x.y1;
        const int kc = (Hh - c0k) / 2 + 1;
        double xp = d.xp, ps = d.ps;
        int kd = d.k;
        if (FIRSTH && own && kd != kc - 1) {
          xp = L.cscr[0];
          ps = L.cscr[1];
          const double kdd = L.cscr[2];
          kd = (kdd == kdd) ? (int)kdd : -1;  // (NaN: nothing pending)
        }
        if (own && kd == kc - 1 && !first) {
          const double r = xp + ((cv - 2.0 * old.y) + ps) * x.c.idy2 - fc.y;
          if (fabs(r) > lc.tol) {
            const int q = L.kmax + kd;
            atomicOr(&L.bits[q >> 6], 1ull << (q & 63));
          }
        }
        if (isc) d.k = -1;
      }
    }
  }
  if (STORE && j >= x.y0 && j < x.y1 && x.out_lane) {
    double2* dst = reinterpret_cast<double2*>(x.pout + (size_t)(j - x.g.row_lo) * (size_t)x.g.pitch + x.gi);
    typedef double d2v __attribute__((ext_vector_type(2)));
    d2v mv = {m.x, m.y};
    __builtin_nontemporal_store(mv, reinterpret_cast<d2v*>(dst));
  }
  if constexpr (!RES || UP) return;
  const bool rrow = j >= x.y0 && j < x.y1 && j >= x.g.j0 && j <= lc.jr1;  // row-uniform
  const double thr = rrow ? lc.tol : __builtin_huge_val();
  const bool row1 = RC && j == 1;  // S is the bottom ghost: the cell's own value stands in
  bool ex;
  if constexpr (A) {  // the other colour at gi+1: W = gi (old; the left ghost when gi+1 == 1), E = gi+2 (new)
    const double pc = m.y;
    double pW = (EDGE && x.gi == 0) ? pc : old.x;
    if constexpr (STEP) pW = (rs == 2 && cc.sa == 1) ? 0.0 + pc : pW;  // W = the step-column solid
    const double pS = row1 ? pc : sb.y;
    const double pE = dpp_from_right(m.x);
    ex = fabs(residual_at<CASE>(x.c, 0, 0, 0, 0, pc, pW, pE, pS, nb.y, fc.y)) > thr;
    if constexpr (EDGE) ex = ex && cc.kb == 3;
    if constexpr (STEP) {
      ex = ex && (rs == 0 || cc.sb == 2);  // fluid cells only
      if (rowc && cc.sb == 1) {  // the corner's south neighbour: its p_N is not known yet (deferred)
        ex = false;
        bool on = true;
        if constexpr ((MODE & LX_ACT) != 0) on = act.c;
        if (FULL && on) {
          d.xp = (pE - 2.0 * pc + pW) * x.c.idx2;
          d.ps = pS;
          d.k = (Hh - 1 - c0k) / 2 + 1;
          if (LASTH && x.out_lane && rrow) {
            L.cscr[0] = d.xp;
            L.cscr[1] = d.ps;
            L.cscr[2] = (double)d.k;
          }
        }
      }
    }
    if constexpr ((MODE & LX_ACT) != 0) ex = ex && act.c;
  } else {  // the other colour at gi: W = gi-1 (old; gi is even, never column 1), E = gi+1 (new)
    const double pc = m.x;
    double pW = dpp_from_left(old.y);
    if constexpr (STEP) pW = (rs == 2 && cc.sa == 2 && x.gi == x.c.step_i + 1) ? 0.0 + pc : pW;
    const double pS = row1 ? pc : sb.x;
    const double pE = m.y;
    ex = fabs(residual_at<CASE>(x.c, 0, 0, 0, 0, pc, pW, pE, pS, nb.x, fc.x)) > thr;
    if constexpr (EDGE) ex = ex && cc.ka == 3;
    if constexpr (STEP) {
      ex = ex && (rs == 0 || cc.sa == 2);
      if (rowc && cc.sa == 1) {
        ex = false;
        bool on = true;
        if constexpr ((MODE & LX_ACT) != 0) on = act.b;
        if (FULL && on) {
          d.xp = (pE - 2.0 * pc + pW) * x.c.idx2;
          d.ps = pS;
          d.k = (Hh - 1 - c0k) / 2 + 1;
          if (LASTH && x.out_lane && rrow) {
            L.cscr[0] = d.xp;
            L.cscr[1] = d.ps;
            L.cscr[2] = (double)d.k;
          }
        }
      }
    }
    if constexpr ((MODE & LX_ACT) != 0) ex = ex && act.b;
  }
  exi = ex ? 1 : exi;
  asm volatile("" : "+v"(exi));
}

// Sampled residuals (MODE & LX_SAMPLE): the loop goes on iff SOME cell's
// residual exceeds tol, so the exact residual of a subset of the cells proves
// "go on" whenever one of them exceeds it. A sampled march evaluates the rows
// j = Rbeg - 10q only: at step T of the 10-step unroll (front row R = Rbeg - T
// - 10q) that is the row at X = T behind the front, a compile-time choice (one
// residual row per step for T = 1 .. 2NS, none otherwise). An iteration whose
// sampled rows all meet the tolerance is left open (LexCtl::kexact, stop
// code 2) and evaluated exactly by the host (Solver::solve_lexw).
template <int MODE, int T, int X>
constexpr bool lx_res_row() { return !(MODE & LX_SAMPLE) || T == X; }

// column data of a wave: the cavity's wall kinds (LxCol) / the open cases' ghost kinds (LxoCol)
template <int CASE>
struct LxCols {
  LxCol cc[2];
  LxoCol oc;
};

template <int CASE, int S, int NS, int T, int ROT, int PAR, int MODE, bool EDGE, bool RC, bool UP = false>
__device__ __forceinline__ void lx_sweeps(const WaveCtx<CAVITY>& x, const LexCtx& lc, const LexCtl& L,
                                          const LxCols<CASE>& cl, LexRun<NS>& s, int R, const LxAct& act, int& exi) {
  if constexpr (S < NS) {
    // red at R+2S+1 (parity PAR^1) in half-sweep H0+2S; black at R+2S+2 (PAR) in H0+2S+1
    // (UP: at R-2S-1, R-2S-2, the same parities)
    constexpr int D = UP ? -1 : 1;
    if constexpr (CASE == CAVITY) {
      lx_row<ROT, PAR ^ 1, 0, MODE, EDGE, false, lx_res_row<MODE, T, 2 * S + 1>(), UP>(
          x, lc, cl.cc, s.w[S], R + D * (2 * S + 1), 2 * S + 1, act, s.fr[LX_S10(2 * S + 1)], exi);
      lx_row<ROT, PAR, 1, MODE, EDGE, S == NS - 1, lx_res_row<MODE, T, 2 * S + 2>(), UP>(
          x, lc, cl.cc, s.w[S], R + D * (2 * S + 2), 2 * S + 2, act, s.fr[LX_S10(2 * S + 2)], exi);
    } else {
      lxo_row<CASE, ROT, PAR ^ 1, 0, MODE, EDGE, RC, false, lx_res_row<MODE, T, 2 * S + 1>(), S == 0, false, UP>(
          x, lc, L, cl.oc, s.w[S], R + D * (2 * S + 1), 2 * S + 1, act, s.fr[LX_S10(2 * S + 1)], exi, s.d);
      double2* nxt = nullptr;  // row R+2S+3 in the next sweep's ring (the step's corner write)
      if constexpr (S + 1 < NS && !UP) nxt = &s.w[S + 1][LX_SLOT(2 * S + 3)];
      lxo_row<CASE, ROT, PAR, 1, MODE, EDGE, RC, S == NS - 1, lx_res_row<MODE, T, 2 * S + 2>(), false, S == NS - 1, UP>(
          x, lc, L, cl.oc, s.w[S], R + D * (2 * S + 2), 2 * S + 2, act, s.fr[LX_S10(2 * S + 2)], exi, s.d, nxt);
    }
    if constexpr (S + 1 < NS) s.w[S + 1][LX_SLOT(2 * S + 2)] = s.w[S][LX_SLOT(2 * S + 2)];
    lx_sweeps<CASE, S + 1, NS, T, ROT, PAR, MODE, EDGE, RC, UP>(x, lc, L, cl, s, R, act, exi);
  }
}

template <int CASE, int NS, int T, int ROT, int PAR, int MODE, bool EDGE, bool RC, bool UP = false>  // PAR = parity of R, T = step of the unroll
__device__ __forceinline__ void lx_step(const WaveCtx<CAVITY>& x, const LexCtx& lc, const LexCtl& L,
                                        const LxCols<CASE>& cl, LexRun<NS>& s, int R, unsigned long long bit) {
  constexpr int D = UP ? -1 : 1;
  s.w[0][LX_SLOT(0)] = s.np[LX_SLOT(0)];
  s.fr[LX_S10(1)] = s.nf[LX_SLOT(0)];
  s.np[LX_SLOT(-4)] = lx_ld(x, x.pin, R - 4 * D);
  s.nf[LX_SLOT(-4)] = lx_ld(x, x.f, R - 3 * D);
  int exi = 0;
  const LxAct act = lx_act<MODE, CASE == BACKSTEP && EDGE && RC>(lc, x.gi, R);
  lx_sweeps<CASE, 0, NS, T, ROT, PAR, MODE, EDGE, RC, UP>(x, lc, L, cl, s, R, act, exi);
  if constexpr (UP) return;  // (no residuals marching up)
  if constexpr ((MODE & LX_SAMPLE) && (T < 1 || T > 2 * NS)) return;  // (no residual row at this step)
  s.mask |= exi ? bit : 0ull;
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

// OR `len` bits (b[0..2], 192 max) into shard `sh` of the bitset at bit q0 >= 0
__device__ __forceinline__ void lexw_flush(const LexCtl& L, int sh, int q0, const unsigned long long (&b)[3], int len) {
  unsigned long long* G = L.bits + (size_t)sh * L.words;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    if (c * 64 >= len || b[c] == 0) continue;
    const int q = q0 + c * 64;
    const int w = q >> 6, o = q & 63;
    if (w < L.words) atomicOr(&G[w], b[c] << o);
    if (o && w + 1 < L.words) atomicOr(&G[w + 1], b[c] >> (64 - o));
  }
}

// UP (the cavity's steady interior bands, lexw_updown): the same march
// mirrored - the front row climbs from below the band, sweep S red at R-2S-1,
// black at R-2S-2 - without residuals (a residual needs its row's south
// neighbour before and north neighbour after a half-sweep: marching up that
// would hold rows for a step longer; the down bands' sampled rows prove the
// iterations). Neighbouring bands marching in opposite directions read their
// shared halo rows at the same time (both at the start or both at the end of
// the launch): they come from L2 instead of HBM twice.
template <int CASE, int NS, int MODE, bool EDGE, bool RC = false, bool UP = false>
__device__ __forceinline__ void lx_march(const WaveCtx<CAVITY>& x, const LexCtx& lc, const LexCtl& L, int y0, int y1,
                                         int c0, int lane, int shard) {
  static_assert(!UP || (!(MODE & LX_ACT) && !EDGE && !RC), "upward march: the unmasked, unchecked interior bands");
  constexpr int H = 2 * NS + 1;
  constexpr int D = UP ? -1 : 1;
  const int Rb0 = UP ? y0 - H : y1 - 1 + H;
  const int Rbeg = UP ? Rb0 - (Rb0 & 1) : Rb0 + (Rb0 & 1);  // even first front row: compile-time colours
  const int nsteps = (y1 - y0) + 2 * H + (Rb0 & 1);
  LexRun<NS> s;
  const double2 z = make_double2(0.0, 0.0);
#pragma unroll
  for (int k = 0; k < 5; ++k)
#pragma unroll
    for (int q = 0; q < NS; ++q) s.w[q][k] = z;
#pragma unroll
  for (int k = 0; k < 10; ++k) s.fr[k] = z;
  {
    constexpr int ROT = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      s.np[LX_SLOT(-q)] = lx_ld(x, x.pin, Rbeg - D * q);
      s.nf[LX_SLOT(-q)] = lx_ld(x, x.f, Rbeg - D * (q - 1));
    }
  }
  s.mask = 0ull;
  s.d = LxDefer{0.0, 0.0, -1};
  LxCols<CASE> cl;
  if constexpr (EDGE && CASE == CAVITY) cl.cc[0] = lx_col(x, x.gi), cl.cc[1] = lx_col(x, x.gi + 1);
  if constexpr (EDGE && CASE != CAVITY)
    cl.oc = LxoCol{lxo_kind(x, x.gi), lxo_kind(x, x.gi + 1), lxs_class(x, x.gi), lxs_class(x, x.gi + 1)};
  int R = Rbeg;
  if constexpr (UP) {
    for (int st = 0; st < nsteps; st += 10, R += 10) {
      lx_step<CASE, NS, 0, 0, 0, MODE, EDGE, RC, true>(x, lc, L, cl, s, R, 0ull);
      lx_step<CASE, NS, 1, 1, 1, MODE, EDGE, RC, true>(x, lc, L, cl, s, R + 1, 0ull);
      lx_step<CASE, NS, 2, 2, 0, MODE, EDGE, RC, true>(x, lc, L, cl, s, R + 2, 0ull);
      lx_step<CASE, NS, 3, 3, 1, MODE, EDGE, RC, true>(x, lc, L, cl, s, R + 3, 0ull);
      lx_step<CASE, NS, 4, 4, 0, MODE, EDGE, RC, true>(x, lc, L, cl, s, R + 4, 0ull);
      lx_step<CASE, NS, 5, 0, 1, MODE, EDGE, RC, true>(x, lc, L, cl, s, R + 5, 0ull);
      lx_step<CASE, NS, 6, 1, 0, MODE, EDGE, RC, true>(x, lc, L, cl, s, R + 6, 0ull);
      lx_step<CASE, NS, 7, 2, 1, MODE, EDGE, RC, true>(x, lc, L, cl, s, R + 7, 0ull);
      lx_step<CASE, NS, 8, 3, 0, MODE, EDGE, RC, true>(x, lc, L, cl, s, R + 8, 0ull);
      lx_step<CASE, NS, 9, 4, 1, MODE, EDGE, RC, true>(x, lc, L, cl, s, R + 9, 0ull);
    }
    return;
  }
  // (nsteps + 9 <= 127 by the host's band limit: bits t/2 < 64)
#define LX_BIT(T) ((((st + (T)) >> 1) < 64) ? (1ull << ((st + (T)) >> 1)) : 0ull)
  for (int st = 0; st < nsteps; st += 10, R -= 10) {
#if CFD_LEXW_GROUPS
    if constexpr (RC && !EDGE && CASE == CHANNEL) {
      // a group of 10 steps whose updated rows (R-8 .. R+2NS) avoid the ghost
      // rows, row 1 (its residual reads the bottom ghost's stand-in) and the
      // stored strip's edge rows runs the unchecked rows (row kinds all
      // interior: the same operations), as open.hip's marches do: the
      // channel's row-checked bands otherwise take ~3x a safe band's time per
      // step and set its launch (34.8 -> 30.9 us, 169 -> 181 GLUPS; the
      // step measured 116.5 -> 114.4 and keeps them checked:
      // profiles/r4_lexw_stamps)
      if (R - 8 >= 2 && R - 8 > x.rmin && R + 2 * NS < lc.jg && R + 2 * NS < x.rmax) {
        lx_step<CASE, NS, 0, 0, 0, MODE, EDGE, false>(x, lc, L, cl, s, R, LX_BIT(0));
        lx_step<CASE, NS, 1, 1, 1, MODE, EDGE, false>(x, lc, L, cl, s, R - 1, LX_BIT(1));
        lx_step<CASE, NS, 2, 2, 0, MODE, EDGE, false>(x, lc, L, cl, s, R - 2, LX_BIT(2));
        lx_step<CASE, NS, 3, 3, 1, MODE, EDGE, false>(x, lc, L, cl, s, R - 3, LX_BIT(3));
        lx_step<CASE, NS, 4, 4, 0, MODE, EDGE, false>(x, lc, L, cl, s, R - 4, LX_BIT(4));
        lx_step<CASE, NS, 5, 0, 1, MODE, EDGE, false>(x, lc, L, cl, s, R - 5, LX_BIT(5));
        lx_step<CASE, NS, 6, 1, 0, MODE, EDGE, false>(x, lc, L, cl, s, R - 6, LX_BIT(6));
        lx_step<CASE, NS, 7, 2, 1, MODE, EDGE, false>(x, lc, L, cl, s, R - 7, LX_BIT(7));
        lx_step<CASE, NS, 8, 3, 0, MODE, EDGE, false>(x, lc, L, cl, s, R - 8, LX_BIT(8));
        lx_step<CASE, NS, 9, 4, 1, MODE, EDGE, false>(x, lc, L, cl, s, R - 9, LX_BIT(9));
        continue;
      }
    }
#endif
    lx_step<CASE, NS, 0, 0, 0, MODE, EDGE, RC>(x, lc, L, cl, s, R, LX_BIT(0));
    lx_step<CASE, NS, 1, 1, 1, MODE, EDGE, RC>(x, lc, L, cl, s, R - 1, LX_BIT(1));
    lx_step<CASE, NS, 2, 2, 0, MODE, EDGE, RC>(x, lc, L, cl, s, R - 2, LX_BIT(2));
    lx_step<CASE, NS, 3, 3, 1, MODE, EDGE, RC>(x, lc, L, cl, s, R - 3, LX_BIT(3));
    lx_step<CASE, NS, 4, 4, 0, MODE, EDGE, RC>(x, lc, L, cl, s, R - 4, LX_BIT(4));
    lx_step<CASE, NS, 5, 0, 1, MODE, EDGE, RC>(x, lc, L, cl, s, R - 5, LX_BIT(5));
    lx_step<CASE, NS, 6, 1, 0, MODE, EDGE, RC>(x, lc, L, cl, s, R - 6, LX_BIT(6));
    lx_step<CASE, NS, 7, 2, 1, MODE, EDGE, RC>(x, lc, L, cl, s, R - 7, LX_BIT(7));
    lx_step<CASE, NS, 8, 3, 0, MODE, EDGE, RC>(x, lc, L, cl, s, R - 8, LX_BIT(8));
    lx_step<CASE, NS, 9, 4, 1, MODE, EDGE, RC>(x, lc, L, cl, s, R - 9, LX_BIT(9));
  }
#undef LX_BIT
  // lane l's bit u <-> iteration Bd0 + u - l = (Bd0 - 63) + (u + 63 - l):
  // shift each lane's mask by 63 - l into a 128-bit run and OR the lanes
  const unsigned long long m = x.out_lane ? s.mask : 0ull;
  const int sh = 63 - lane;
  const unsigned long long lo = m << sh, hi = sh ? (m >> (64 - sh)) : 0ull;
  unsigned long long b[3] = {wave_or64(lo), wave_or64(hi), 0ull};
  const int Bd0 = (lc.H0 - c0 - Rbeg - 2) / 2 + 1;
  if (lane == 0) lexw_flush(L, shard, Bd0 - 63 + L.kmax, b, 128);
}

// Owned rows of column tile `ct` whose output cells launch H0 touches: a cell
// (j,i) is updated in one of the launch's half-sweeps or has its black
// residual of half-sweep H0-1 evaluated (i+j <= H0+2NS-1 and i+j+2(K-1) >=
// H0-1), or finished in the previous launch and must be copied into this
// launch's output buffer (i+j+2(K-1) >= H0-2NS). Other rows hold their final
// values in both buffers already.
// Open cases: the ghost rows / columns too, the left / bottom ghosts active two
// half-sweeps later than their position (lxo_row).
__host__ __device__ inline void lexw_rows(const Geo& g, int H0, int K, int ns, int ct, int* lo, int* hi,
                                          bool open = false) {
  const int twc = lexw_twc(ns);
  if (!open) {
    const int cmin = max(ct * twc, 1), cmax = min(ct * twc + twc - 1, g.nx);
    *lo = max(g.j0, H0 - 2 * ns - 2 * (K - 1) - cmax);
    *hi = min(g.j1, H0 + 2 * ns - 1 - cmin);
  } else {
    const int cmin = max(ct * twc, 0), cmax = min(ct * twc + twc - 1, g.nx + 1);
    *lo = max(g.wj0, H0 - 2 * ns - 2 * (K - 1) - cmax - 2);
    *hi = min(g.wj1, H0 + 2 * ns - 1 - cmin);
  }
}

// diagnostic build only (CFD_LEXW_STAMPS=1, never the product library): per
// launch (H0 / 2NS) and march path (0 wall tiles, 1 unmasked, 2 masked, 3
// steady interior, 4 the step's block-crossing tiles on the masked march or
// the cavity's steady interior bands marching up, 5
// the step's left tiles, 6 / 7 row-checked open-case ramp / steady) the maximum and the
// sum of the waves' march cycles and the wave count (solver.hip
// cfd_lexw_stamps, scripts/dbg/lexw_stamps.py)
#ifndef CFD_LEXW_STAMPS
#define CFD_LEXW_STAMPS 0
#endif
#if CFD_LEXW_STAMPS
constexpr int LEXW_STAMP_LAUNCHES = 8192;
static __device__ unsigned long long lexw_stamp_buf[LEXW_STAMP_LAUNCHES * 8 * 3];
// per wave of the launches li = LEXW_WSTAMP_L0 .. +LEXW_WSTAMP_N-1: {cycles, start
// memtime, ctile << 32 | y0, xcc id}, by tile (is a slow wave slow in every launch?)
#ifndef LEXW_WSTAMP_L0
#define LEXW_WSTAMP_L0 1500
#endif
constexpr int LEXW_WSTAMP_N = 8, LEXW_WSTAMP_T = 4096;
static __device__ unsigned long long lexw_wstamp_buf[LEXW_WSTAMP_N * LEXW_WSTAMP_T * 4];
#endif

// One launch of NS lexicographic-order sweeps (half-sweeps H0 .. H0+2NS-1) on
// one strip, tiled as poisson_multi_kernel (PairPlan). RAMP = false: a launch
// in which every cell is active in every half-sweep (no activity masks: 4
// waves per SIMD); RAMP = true: the launches at the start and the end of the
// solve, whose tiles take the masked marches unless wholly active (the masked
// code would cost the steady kernel registers, so it lives in its own kernel).
template <int CASE, int NS, bool RAMP, bool SAMPLE = false>
__global__ __launch_bounds__(256, RAMP ? 2 : CFD_LEXW_MIN_WAVES(NS)) void poisson_lexw_kernel(Geo g, Coef c, const double* __restrict__ pin,
                                                              double* __restrict__ pout, const double* __restrict__ f,
                                                              LexCtl L, int H0, int K, int ka, int kb, PairPlan pl,
                                                              int flags, LexRamp rp) {
  static_assert(CASE == CAVITY || CASE == CHANNEL || CASE == BACKSTEP, "reference-order march: case");
  constexpr bool OPEN = CASE != CAVITY;
  constexpr int CH = lexw_ch(NS);  // left column halo (lanes 0 .. CH/2-1)
  constexpr int H = 2 * NS + 1;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (!(flags & 4) && !lexw_go_on(L, ka, kb, blockIdx.x == 0 && wv == 0, lane)) return;

  const int nblk = (int)gridDim.x;
  const int L8 = (nblk / 8) * 8;
  const int bl = (int)blockIdx.x;
#ifndef CFD_LEXW_XCD_ROT
#define CFD_LEXW_XCD_ROT 0  // (diagnostic A/B: rotate which XCD marches which range of tiles)
#endif
  const int blk = (bl < L8) ? ((bl + CFD_LEXW_XCD_ROT) % 8) * (nblk / 8) + bl / 8 : bl;
  const int tile = blk * 4 + wv;
  int ctile, y0, y1;
  // (flags bit 4: the cavity's odd bands march up where the tile is wholly
  // active - steady launches, and the ramp launches' full interior tiles)
  bool up = false;
  if (rp.nb > 0) {  // ramp launch (LexRamp): binary search of the tile's band
    int lo = 0, hi = rp.nb - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if ((int)(rp.band[mid] >> 16) <= tile) lo = mid;
      else hi = mid - 1;
    }
    const unsigned e = rp.band[lo];
    const int ca = (e >> 8) & 255, cb = e & 255;
    // wall tiles (masked march, slower per step; they set the ramp launches'
    // time) and the step's crossing tiles at the block's edge: two waves each,
    // one per half band (host: launch_lexw build)
    int half;
    lexw_ramp_waves(rp, pl.ctiles, lo, ca, cb, tile - (int)(e >> 16), &ctile, &half);
    if (ctile > cb) return;
    up = (lo & 1) && (flags & 16) && half < 0;
    int rlo, rhi;
    lexw_rows(g, H0, K, NS, ctile, &rlo, &rhi, OPEN);
    y0 = max(rp.row0 + lo * rp.th, rlo);
    y1 = min(rp.row0 + (lo + 1) * rp.th, rhi + 1);
    if (half >= 0) {
      const int mid = rp.row0 + lo * rp.th + rp.th / 2;
      if (half == 0) y1 = min(y1, mid);
      else y0 = max(y0, mid);
    }
  } else {
    const int ne = (pl.ctiles >= 2) ? 2 : 1;
    const int nbe = pl.nbe0 + pl.nbe1, nbi = pl.nb0 + pl.nb1;
    int band, th, nb0, part = -1;
    if (tile < ne * nbe) {
      ctile = (tile < nbe) ? 0 : pl.ctiles - 1;
      band = tile % nbe;
      th = pl.the;
      nb0 = pl.nbe0;
    } else {
      const int t = tile - ne * nbe;
      const int nci = pl.ctiles - ne;
      if (t < nci * nbi) {
        ctile = 1 + t % nci;
        band = t / nci;
        // (the step's split bands: part 0 here, the others below)
        if (ctile - pl.xa < pl.xn && ctile >= pl.xa && band - pl.xb < pl.xbn && band >= pl.xb) part = 0;
        up = (band & 1) && (flags & 16);
      } else {
        const int u = t - nci * nbi, nx = pl.xn * pl.xbn;
        if (u >= nx * (pl.xparts - 1)) return;
        const int v = u % nx;
        part = 1 + u / nx;
        ctile = pl.xa + v % pl.xn;
        band = pl.xb + v / pl.xn;
      }
      th = pl.th;
      nb0 = pl.nb0;
    }
    const bool r0 = band < nb0;
    y0 = r0 ? pl.lo0 + band * th : pl.lo1 + (band - nb0) * th;
    y1 = min(y0 + th, r0 ? pl.hi0 : pl.hi1);
    if (part >= 0) {
      const int len = y1 - y0;
      y1 = y0 + len * (part + 1) / pl.xparts;
      y0 = y0 + len * part / pl.xparts;
    }
  }
  constexpr int TWC = lexw_twc(NS);
  const int c0 = ctile * TWC - CH;
  const int gi = c0 + 2 * lane;
  // backwards step: a column tile whose march columns all lie left of the
  // step's column (the first wall tile included) sees the block's rows jb ..
  // ny as row-uniform rules: its bottom row jb refreshed as 0.0 + p_S, the
  // rows above it interior solids that never change, and their ghosts (the
  // top ghost row, the left ghost column above jb) constants the host set
  // before the solve (Solver::lexw_presolid). Its bands end at row jb: the
  // left tiles march as a channel whose top ghost row is jb (lxo_row,
  // LexCtx::jg), with no per-cell solid rules.
  bool left = false;
  if constexpr (CASE == BACKSTEP) {
    if (c0 + 127 <= c.step_i - 1 && (flags & 8)) {  // (flags bit 3: the host set those ghosts)
      left = c0 >= 1;
      y1 = min(y1, c.inlet_jmax + 2);
    }
  }
  if (y0 >= y1) return;

  // activity of the marched region (rows y0-H-1 .. y1+H, columns c0 .. c0+127,
  // interior cells; open cases: ghosts too, the left / bottom ones two
  // half-sweeps late) over this launch's half-sweeps (and the previous
  // launch's last one, whose black residuals this launch evaluates)
  constexpr int GLO = OPEN ? 0 : 1;  // lowest row / column index with cells that change
  const int rlo = max(max(y0 - H - 1, GLO), g.row_lo);
  const int rhi = min(min(y1 + H, g.ny + 1 - GLO), g.row_lo + g.nrows - 1);
  const int clo = max(c0, GLO), chi = min(c0 + 127, g.nx + 1 - GLO);
  const int smin = clo + rlo, smax = chi + rhi;
  const int Hend = H0 + 2 * NS - 1;
  const int last = 2 * (K - 1) + (OPEN ? 2 : 0);
  if (smin > Hend) return;                // not started: both buffers hold the initial field
  if (smax + last < H0 - 2 * NS) return;  // finished before the previous launch: both hold the result
  const bool cols_in = OPEN ? (c0 >= 1 && c0 + 127 <= g.nx) : (clo == c0 && chi == c0 + 127);

  WaveCtx<CAVITY> x{g, c};
  x.pin = pin; x.pout = pout; x.f = f;
  x.gi = gi;
  x.y0 = y0;
  x.y1 = y1;
  x.rmin = max(g.row_lo, 0);
  x.rmax = min(g.row_lo + g.nrows - 1, g.ny + 1);
  x.pair_ok = gi >= 0 && gi + 1 < g.pitch;
  x.out_lane = x.pair_ok && lane >= CH / 2 && lane < CH / 2 + TWC / 2;
  x.icol_a = gi >= 1 && gi <= g.nx;
  x.icol_b = gi + 1 >= 1 && gi + 1 <= g.nx;
  x.open_a = x.open_b = true;
  x.gic = min(max(gi, 0), g.pitch - 2);
  // (readfirstlane: opaque wave-uniform values, so selects between them stay
  // selects of values)
  auto uni = [](double v) {
    return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)),
                            __builtin_amdgcn_readfirstlane(__double2loint(v)));
  };
  LexCtx lc{H0, K, L.tol[0], uni(c.om_nc[2]), uni(c.om_nc[3]), uni(c.om_nc[4]),
            left ? c.inlet_jmax + 1 : g.ny + 1, left ? min(g.j1, c.inlet_jmax) : g.j1, left ? 0.0 : -0.0};
  if (left) x.rmax = min(x.rmax, c.inlet_jmax + 2);  // (rows above jb: kept; loads clamped there)
  const int shard = bl & (LEXW_SHARDS - 1);
  const bool edge = !cols_in;
  constexpr int SM = SAMPLE ? LX_SAMPLE : 0;
#if CFD_LEXW_STAMPS
  long long t0_;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0_)::"memory");
  int path_ = 0;
#define LX_PATH(v) (path_ = (v))
#else
#define LX_PATH(v) ((void)0)
#endif
  if constexpr (!OPEN) {
    if constexpr (RAMP) {
      // tiles of a ramp launch whose every cell is active in every half-sweep
      // it evaluates (H0-1 .. H0+2NS-1) take the unmasked march
      const bool full = smax <= H0 - 2 && Hend <= smin + last;
      // (wall tiles too: a wholly active one takes the steady launches' edge
      // march, not the masked one - the masked wall marches set the ramps' time)
      if (edge && full && CFD_LEXW_RAMP_EDGE_FULL) { LX_PATH(0); lx_march<CASE, NS, SM, true>(x, lc, L, y0, y1, c0, lane, shard); }
      else if (edge) { LX_PATH(0); lx_march<CASE, NS, LX_ACT | SM, true>(x, lc, L, y0, y1, c0, lane, shard); }
      else if (full && SAMPLE && up) { LX_PATH(1); lx_march<CASE, NS, SM, false, false, SAMPLE>(x, lc, L, y0, y1, c0, lane, shard); }
      else if (full) { LX_PATH(1); lx_march<CASE, NS, SM, false>(x, lc, L, y0, y1, c0, lane, shard); }
      else { LX_PATH(2); lx_march<CASE, NS, LX_ACT | SM, false>(x, lc, L, y0, y1, c0, lane, shard); }
    } else {
      if (edge) { LX_PATH(0); lx_march<CASE, NS, SM, true>(x, lc, L, y0, y1, c0, lane, shard); }
      else if (SAMPLE && up) { LX_PATH(4); lx_march<CASE, NS, SM, false, false, SAMPLE>(x, lc, L, y0, y1, c0, lane, shard); }
      else { LX_PATH(3); lx_march<CASE, NS, SM, false>(x, lc, L, y0, y1, c0, lane, shard); }
    }
  } else {
    // row checks unless every row the march updates (y0-H+1 .. y1+H+2NS) lies
    // strictly between the stored strip's edge rows (ghost rows included)
    bool rc = CFD_LEXW_ALLRC || !(y0 - H + 1 > x.rmin && y1 + H + 2 * NS < min(x.rmax, lc.jg));
    bool edge_ = edge;
    if (CASE == BACKSTEP && !left) {
      const int jb = c.inlet_jmax + 1, si = c.step_i;
      // a march over interior solids only (rows y0-H-1 .. y1+H+2NS+1 in jb+1 ..
      // ny, columns in 1 .. si-1): nothing it touches ever changes
      if (c0 >= 1 && c0 + 127 <= si - 1 && y0 - H - 1 >= jb + 1 && y1 + H + 2 * NS + 1 <= g.ny) return;
      // a march reaching the block (rows >= jb-1, columns <= si+1): the general
      // tiles (per-cell solid rules, lxo_row STEP)
      if (y1 + H + 2 * NS + 1 >= jb - 1 && c0 <= si + 1) rc = edge_ = true;
    }
    const bool edge = edge_;
    if constexpr (RAMP) {
      const bool full = !rc && smax <= H0 - 2 && Hend <= smin + 2 * (K - 1);
      // an edge march (ghosts, the step's solids) wholly active in every
      // half-sweep it evaluates, the left / bottom ghosts and the step-column
      // solids two half-sweeps late included: the steady launches' edge march
      const bool efull = smax + 2 <= H0 - 2 && Hend <= smin + 2 * (K - 1);
      if (edge && efull && CFD_LEXW_RAMP_EDGE_FULL) {
        LX_PATH(0);
        lx_march<CASE, NS, SM, true, true>(x, lc, L, y0, y1, c0, lane, shard);
      } else if (edge) { LX_PATH(0); lx_march<CASE, NS, LX_ACT | SM, true, true>(x, lc, L, y0, y1, c0, lane, shard); }
      else if (full && SAMPLE && up) { LX_PATH(1); lx_march<CASE, NS, SM, false, false, SAMPLE>(x, lc, L, y0, y1, c0, lane, shard); }
      else if (full) { LX_PATH(1); lx_march<CASE, NS, SM, false, false>(x, lc, L, y0, y1, c0, lane, shard); }
      else if (rc && efull && CFD_LEXW_RAMP_EDGE_FULL) {  // (row-checked bands likewise: the steady rc march)
        LX_PATH(6);
        lx_march<CASE, NS, SM, false, true>(x, lc, L, y0, y1, c0, lane, shard);
      } else if (rc) { LX_PATH(6); lx_march<CASE, NS, LX_ACT | SM, false, true>(x, lc, L, y0, y1, c0, lane, shard); }
      else { LX_PATH(2); lx_march<CASE, NS, LX_ACT | SM, false, false>(x, lc, L, y0, y1, c0, lane, shard); }
    } else {
      if (edge) { LX_PATH(0); lx_march<CASE, NS, SM, true, true>(x, lc, L, y0, y1, c0, lane, shard); }
      else if (rc) { LX_PATH(7); lx_march<CASE, NS, SM, false, true>(x, lc, L, y0, y1, c0, lane, shard); }
      else if (SAMPLE && up) { LX_PATH(3); lx_march<CASE, NS, SM, false, false, SAMPLE>(x, lc, L, y0, y1, c0, lane, shard); }
      else { LX_PATH(3); lx_march<CASE, NS, SM, false, false>(x, lc, L, y0, y1, c0, lane, shard); }
    }
  }
#if CFD_LEXW_STAMPS
  {
    long long t1_;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1_)::"memory");
    const int li = H0 / (2 * NS);
    if (OPEN && path_ == 0 && cols_in) path_ = 4;  // the step's block / crossing tiles on the masked march
    if (left) path_ = 5;                           // the step's left tiles
    if (lane == 0 && li >= 0 && li < LEXW_STAMP_LAUNCHES) {
      unsigned long long* b = lexw_stamp_buf + ((size_t)li * 8 + path_) * 3;
      const unsigned long long cyc = (unsigned long long)(t1_ - t0_);
      atomicMax(b, cyc);
      atomicAdd(b + 1, cyc);
      atomicAdd(b + 2, 1ull);
      const int wl = li - LEXW_WSTAMP_L0;
      if (wl >= 0 && wl < LEXW_WSTAMP_N && tile < LEXW_WSTAMP_T) {
        unsigned long long* w = lexw_wstamp_buf + ((size_t)wl * LEXW_WSTAMP_T + tile) * 4;
        unsigned xcc = 0;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        w[0] = cyc;
        w[1] = (unsigned long long)t0_;
        w[2] = ((unsigned long long)(unsigned)ctile << 32) | (unsigned)y0;
        w[3] = xcc;
      }
    }
  }
#endif
#undef LX_PATH
}

#undef LX_SLOT
#undef LX_S10

// max-norm residual of a cavity field (cavity-01.cpp:659-677) over the owned
// interior cells: the residual the reference reports after its last sweep.
// Column pairs like cavity_source_kernel: a wave covers 128 columns of one
// row with 16-B loads, row neighbours by DPP (lanes 0 / 63 load theirs).
__global__ __launch_bounds__(256) void cavity_resmax_kernel(Geo g, Coef c, const double* __restrict__ p,
                                                            const double* __restrict__ f, double* __restrict__ shards) {
  const int lane = threadIdx.x & 63;
  const int gi = blockIdx.x * 128 + 2 * lane;  // even: 16-B aligned pair
  const int j = max(g.j0, 1) + blockIdx.y * 4 + (threadIdx.x >> 6);
  const int nx = g.nx, ny = g.ny;
  double m = 0.0;
  if (j <= min(g.j1, ny) && gi <= nx) {  // (a lane's left neighbour is active)
    const size_t o = at(g, j, gi), P = (size_t)g.pitch;
    const double2 pc = *reinterpret_cast<const double2*>(p + o);
    const double2 ps = *reinterpret_cast<const double2*>(p + o - P);
    const double2 pn = *reinterpret_cast<const double2*>(p + o + P);
    const double2 fc = *reinterpret_cast<const double2*>(f + o);
    double pw = dpp_from_left(pc.y), pe = dpp_from_right(pc.x);
    if (lane == 0) pw = p[o - 1];
    if (lane == 63 || gi + 2 > nx) pe = p[o + 2];  // (the right neighbour lane idles past nx; o + 2 <= nx + 2 < pitch)
    const double ra = residual_abs<CAVITY>(c, nx, ny, j, gi, pc.x, pw, pc.y, ps.x, pn.x, fc.x);
    const double rb = residual_abs<CAVITY>(c, nx, ny, j, gi + 1, pc.y, pc.x, pe, ps.y, pn.y, fc.y);
    m = fmax(gi >= 1 ? ra : 0.0, gi + 1 <= nx ? rb : 0.0);
  }
  block_max_to_shard<256>(m, shards, (blockIdx.y * gridDim.x + blockIdx.x) % RES_SHARDS);
}

// backwards step, lexicographic order: the corner solid (jb, si) of the final
// field as the reference's last refresh leaves it, ((0.0 + p_E) + p_S) / 2
// (backwards_step-01.cpp:708-738; the march keeps the value its south
// neighbour's last update wrote, one iteration older: lxo_row)
__global__ void step_corner_kernel(Geo g, Coef c, double* __restrict__ p) {
  const int jb = c.inlet_jmax + 1, si = c.step_i;
  if (threadIdx.x != 0 || blockIdx.x != 0 || jb < g.j0 || jb > g.j1) return;
  p[at(g, jb, si)] = ((0.0 + p[at(g, jb, si + 1)]) + p[at(g, jb - 1, si)]) * 0.5;
}

// backwards step, reference order: the ghosts next to the block's interior
// solids - the top ghost row over columns 1 .. si-1 and the left ghost column
// over rows jb+1 .. ny - take the values the reference's first refresh after
// a sweep gives them (backwards_step-01.cpp:688-705: copies of interior
// solids, which never change) before the solve, in both buffers. Nothing
// reads them before that refresh (solids are never updated, residuals cover
// fluid cells only), so the solve's iterates are unchanged, and the march's
// column tiles left of the step's column end at the block's bottom row
// (poisson_lexw_kernel, flags bit 3). Owned rows of the strip; halos follow by
// exchange.
__global__ void step_presolid_kernel(Geo g, Coef c, double* __restrict__ p) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int ny = g.ny, si = c.step_i, jb = c.inlet_jmax + 1;
  if (t >= 1 && t <= si - 1 && g.wj1 == ny + 1) p[at(g, ny + 1, t)] = p[at(g, ny, t)];
  const int j = jb + 1 + t;
  if (j <= ny && j >= g.j0 && j <= g.j1) p[at(g, j, 0)] = p[at(g, j, 1)];
}

// max-norm residual of an open-case field over its fluid cells
// (channel-01.cpp:672-681, backwards_step-01.cpp:916-930), ghosts as stored
// (the final field's are refreshed): the residual the reference reports after
// its last sweep, in lexicographic mode. One cell per thread.
template <int CASE>
__global__ __launch_bounds__(256) void open_resmax_kernel(Geo g, Coef c, const double* __restrict__ p,
                                                          const double* __restrict__ f, double* __restrict__ shards) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63) + 1;
  const int j = max(g.j0, 1) + blockIdx.y * 4 + (threadIdx.x >> 6);
  const int nx = g.nx, ny = g.ny;
  double m = 0.0;
  if (j <= min(g.j1, ny) && i <= nx && is_fluid(c, nx, ny, j, i)) {
    const size_t o = at(g, j, i), P = (size_t)g.pitch;
    m = residual_abs<CASE>(c, nx, ny, j, i, p[o], p[o - 1], p[o + 1], p[o - P], p[o + P], f[o]);
  }
  block_max_to_shard<256>(m, shards, (blockIdx.y * gridDim.x + blockIdx.x) % RES_SHARDS);
}

}  // namespace cfd
