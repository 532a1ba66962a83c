// open.hip — proof-mode red-black SOR launches of the open cases (channel,
// backwards step): four sweeps per launch on the wave march (march.hpp).
//
// The cavity's proof-mode launch (march.hpp cav_march) runs NS sweeps with a
// dependency depth of 2 rows per sweep: red at R-(2S+1)d, black at R-(2S+2)d,
// and that black row is sweep S+1's front row. The open cases add the ghost /
// solid refresh after each sweep (channel-01.cpp:531-541,
// backwards_step-01.cpp:685-740), which would cost a third row per sweep.
// Here every refreshed cell takes its value in the skew instead, from the
// same pre-refresh neighbours the reference uses, without extra depth:
//   * rules reading the cell's own row (ghost columns: p[j][0] = p[j][1],
//     p[j][nx+1] = 0; the step block's right column: 0 + p_E) and rules
//     reading the row the march reached EARLIER (down march: row j-1 - ghost
//     row ny+1 = p[ny], the block's lower edge 0 + p_S, the corner
//     ((0 + p_E) + p_S) / 2; up march: row j+1 - ghost row 0 = p[1]) are
//     applied when the row is copied into sweep S+1's window (it has just had
//     its black update, the earlier row is final);
//   * rules reading the row the march reaches LATER are applied one step
//     later, when that row has had its black update: the row is then at
//     R-(2S+3)d, one behind sweep S+1's red row, so sweep S+1 reads the
//     refreshed value in time;
//   * the last sweep stores each row with every rule applied.
// Sweep S's own window keeps the pre-refresh values (its later black updates
// read them, as the reference's sweep does). The convergence test is the
// proof-mode test (device.hpp proof_ratio_gen with the open
// cases' K = 2 (idx2 + idy2)(1 - w)/w): interior-column waves record
// max |p' - p| over their black cells with four fluid neighbours the refresh
// leaves alone (2 <= i, j <= n-1, none next to the step's block). No residual
// stage, so four sweeps fit the 8-row / 8-column halos. An iteration the proof
// leaves open is evaluated exactly by the host's fallback (pair launches).
// The step's block edge and corner read the fluid row below after the sweep:
// one row deeper than the pipeline, so a strip whose first owned row is that
// edge row needs 2 NS + 1 halo rows - strips and ranks run the step's proof
// launches with 3 sweeps (7 rows), one strip with 4.
#include "march.hpp"
#include "open.hpp"

namespace cfd {

#define CFD_SLOT(X) ((((ROT) + 4 - (X)) % 5 + 10) % 5)
#define CFD_S10(X) ((((6 * (ROT) + 5 * (PAR)) % 10 + 9 - (X)) % 10 + 20) % 10)

template <int NS>
struct OpenRun {
  double2 w[NS][5];  // sweep s: rows R-2s d .. R-(2s+4) d
  double2 fr[10];    // source rows R-d .. R-10d
  double2 np[10];    // prefetched p_in rows (row R - X d in slot CFD_S10(X))
  double2 nf[10];    // prefetched f rows
  double dm[NS];     // max |black update| of the proving cells, per sweep
  double pm;         // max |p_in| over every row this wave loads
};

// lane constants of a boundary-column / block wave (EDGE): which of the two
// columns (slot a: gi, slot b: gi + 1) are grid columns 1..nx, ghost
// columns, the step block's columns and its right column
struct OpenLanes {
  bool ic_a, ic_b;        // 1 <= i <= nx
  bool g0_a;              // slot a is column 0 (slot b is column 1)
  bool gn_a, gn_b;        // column nx + 1
  bool bk_a, bk_b;        // 1 <= i <= step_i (the block's columns)
  bool rc_a, rc_b;        // i == step_i (its right column)
};

template <int CASE>
__device__ __forceinline__ OpenLanes open_lanes(const WaveCtx<CASE>& x) {
  const int nx = x.g.nx, ia = x.gi, ib = x.gi + 1, si = CASE == BACKSTEP ? x.c.step_i : -10;
  OpenLanes L;
  L.ic_a = ia >= 1 && ia <= nx;
  L.ic_b = ib >= 1 && ib <= nx;
  L.g0_a = ia == 0;
  L.gn_a = ia == nx + 1;
  L.gn_b = ib == nx + 1;
  L.bk_a = CASE == BACKSTEP && ia >= 1 && ia <= si;
  L.bk_b = CASE == BACKSTEP && ib >= 1 && ib <= si;
  L.rc_a = CASE == BACKSTEP && ia == si;
  L.rc_b = CASE == BACKSTEP && ib == si;
  return L;
}

// The refresh of row j (value m, its pre-refresh neighbours lo = row j-1, hi
// = row j+1), restricted to PART: 1 = same-row rules + rules reading lo,
// 2 = same-row rules + rules reading hi, 4 = rules reading lo only, 8 = rules
// reading hi only (bit sets: 3 = everything). EDGE: ghost columns and the
// step's block (interior-column waves have neither).
template <int CASE, bool EDGE, int PART>
__device__ __forceinline__ double2 open_refresh(const WaveCtx<CASE>& x, const OpenLanes& L, int j, double2 m,
                                                const double2& lo, const double2& hi) {
  const int ny = x.g.ny;
  constexpr bool SAME = (PART & 3) != 0, USE_LO = (PART & 5) != 0, USE_HI = (PART & 10) != 0;
  if (j == 0) {  // ghost row 0: p[0][i] = p[1][i], 1 <= i <= nx (reads hi)
    if (USE_HI) {
      if (!EDGE) return hi;
      m.x = L.ic_a ? hi.x : m.x;
      m.y = L.ic_b ? hi.y : m.y;
    }
    return m;
  }
  if (j == ny + 1) {  // ghost row ny+1: p[ny+1][i] = p[ny][i] (reads lo)
    if (USE_LO) {
      if (!EDGE) return lo;
      m.x = L.ic_a ? lo.x : m.x;
      m.y = L.ic_b ? lo.y : m.y;
    }
    return m;
  }
  if (!EDGE || j < 1 || j > ny) return m;
  // same row (as the value arrives: post-black, pre-refresh)
  const double Ea = m.y, Eb = dpp_from_right(m.x);  // east neighbours of slots a / b (all lanes active)
  if (SAME) {
    m.x = L.g0_a ? m.y : m.x;     // p[j][0] = p[j][1]
    m.x = L.gn_a ? 0.0 : m.x;     // p[j][nx+1] = 0
    m.y = L.gn_b ? 0.0 : m.y;
  }
  if (CASE == BACKSTEP) {
    const int jb = x.c.inlet_jmax + 1;  // the block's lower edge row
    if (SAME && j > jb) {               // right column: 0 + p_E (backwards_step-01.cpp:708-738)
      m.x = L.rc_a ? 0.0 + Ea : m.x;
      m.y = L.rc_b ? 0.0 + Eb : m.y;
    }
    if (USE_LO && j == jb) {  // lower edge: 0 + p_S; corner: ((0 + p_E) + p_S) / 2
      m.x = L.rc_a ? ((0.0 + Ea) + lo.x) / 2 : L.bk_a ? 0.0 + lo.x : m.x;
      m.y = L.rc_b ? ((0.0 + Eb) + lo.y) / 2 : L.bk_b ? 0.0 + lo.y : m.y;
    }
  }
  return m;
}

// red (COLOR 0) / black (COLOR 1) update of row j = R - X d (row parity JPAR)
// on window W (sweep s). RC: the row may be a ghost row, outside the stored
// rows or (step) a block row; EDGE: per-lane masks. wgt (black, PROOF): 1 on
// rows whose proving cells record |p' - p|.
template <int CASE, int DIR, int ROT, int JPAR, int COLOR, bool EDGE, bool RC>
__device__ __forceinline__ void open_update(const WaveCtx<CASE>& x, const OpenLanes& L, double2 (&W)[5], int j,
                                            int X, const double2& fc, double wgt, double* dm) {
  double2& m = W[CFD_SLOT(X)];
  const double2 bh = W[CFD_SLOT(X + 1)], ah = W[CFD_SLOT(X - 1)];
#define CFD_S(b, a) ((DIR > 0) ? (b) : (a))
#define CFD_N(b, a) ((DIR > 0) ? (a) : (b))
  if (!RC || (j > x.rmin && j < x.rmax && j >= 1 && j <= x.g.ny)) {  // row-uniform
    // step: block rows (j > inlet_jmax) update only the columns right of the block
    const bool brow = CASE == BACKSTEP && EDGE && j > x.c.inlet_jmax;
    if (((JPAR ^ COLOR) & 1) == 0) {  // slot a (even column gi) has this colour
      const double Lb = dpp_from_left(m.y);
      const double nv = sor_interior<CASE>(x.c, m.x, Lb, m.y, CFD_S(bh.x, ah.x), CFD_N(bh.x, ah.x), fc.x);
      const double old = m.x;
      m.x = (!EDGE || (L.ic_a && !(brow && L.bk_a))) ? nv : m.x;
      if (!EDGE && COLOR == 1) *dm = fmax(*dm, fabs(m.x - old) * wgt);
    } else {
      const double Ra = dpp_from_right(m.x);
      const double nv = sor_interior<CASE>(x.c, m.y, m.x, Ra, CFD_S(bh.y, ah.y), CFD_N(bh.y, ah.y), fc.y);
      const double old = m.y;
      m.y = (!EDGE || (L.ic_b && !(brow && L.bk_b))) ? nv : m.y;
      if (!EDGE && COLOR == 1) *dm = fmax(*dm, fabs(m.y - old) * wgt);
    }
  }
#undef CFD_S
#undef CFD_N
}

// rows j - 1 / j + 1 of the row at offset X of window W: the one the march
// reached earlier is X + 1, the later one X - 1
template <int DIR, int ROT>
__device__ __forceinline__ double2 open_lo(const double2 (&W)[5], int X) {
  return (DIR > 0) ? W[CFD_SLOT(X + 1)] : W[CFD_SLOT(X - 1)];
}
template <int DIR, int ROT>
__device__ __forceinline__ double2 open_hi(const double2 (&W)[5], int X) {
  return (DIR > 0) ? W[CFD_SLOT(X - 1)] : W[CFD_SLOT(X + 1)];
}

template <int S, int NS, int CASE, int DIR, int ROT, int PAR, bool EDGE, bool RC>
__device__ __forceinline__ void open_sweeps(const WaveCtx<CASE>& x, const OpenLanes& L, OpenRun<NS>& s, int R) {
  if constexpr (S < NS) {
    const int jr = R - (2 * S + 1) * DIR, jb = R - (2 * S + 2) * DIR;
    open_update<CASE, DIR, ROT, PAR ^ 1, 0, EDGE, RC>(x, L, s.w[S], jr, 2 * S + 1, s.fr[CFD_S10(2 * S + 1)], 0.0,
                                                      nullptr);
    // proving rows: band output rows, 2 <= j <= ny - 1 (py0 / py1); the
    // step's interior-column waves lie right of the block's neighbours
    const double wgt = (jb >= x.py0 && jb < x.py1) ? 1.0 : 0.0;  // row-uniform
    open_update<CASE, DIR, ROT, PAR, 1, EDGE, RC>(x, L, s.w[S], jb, 2 * S + 2, s.fr[CFD_S10(2 * S + 2)], wgt,
                                                  &s.dm[S]);
    if constexpr (S + 1 < NS) {
      // row jb (just final for sweep S) into sweep S+1's window, refreshed by
      // its own row and the row reached earlier (lo on the down march)
      double2 v = s.w[S][CFD_SLOT(2 * S + 2)];
      if (RC || EDGE)  // (EDGE without RC: the same-row rules of the ghost columns / block column)
        v = open_refresh<CASE, EDGE, (DIR > 0) ? 1 : 2>(x, L, jb, v, open_lo<DIR, ROT>(s.w[S], 2 * S + 2),
                                                        open_hi<DIR, ROT>(s.w[S], 2 * S + 2));
      s.w[S + 1][CFD_SLOT(2 * S + 2)] = v;
      // the row behind it (reached earlier, already in sweep S+1's window):
      // its rules reading row jb (hi on the down march)
      if (RC) {
        const int jp = jb - DIR;
        double2& t = s.w[S + 1][CFD_SLOT(2 * S + 3)];
        const double2 own = s.w[S][CFD_SLOT(2 * S + 3)];  // pre-refresh (E of the corner)
        const double2 fin = s.w[S][CFD_SLOT(2 * S + 2)];  // row jb, final
        const double2 r = open_refresh<CASE, EDGE, (DIR > 0) ? 8 : 4>(x, L, jp, own, fin, fin);
        // only the cells those rules refresh change (the others keep t)
        if (DIR > 0) {
          if (jp == 0) t = EDGE ? make_double2(L.ic_a ? r.x : t.x, L.ic_b ? r.y : t.y) : r;
        } else {
          if (jp == x.g.ny + 1) t = EDGE ? make_double2(L.ic_a ? r.x : t.x, L.ic_b ? r.y : t.y) : r;
          if (CASE == BACKSTEP && EDGE && jp == x.c.inlet_jmax + 1)
            t = make_double2(L.bk_a ? r.x : t.x, L.bk_b ? r.y : t.y);
        }
      }
    } else {
      // the last sweep stores row R - (2NS+1)d with every rule applied
      const int js = R - (2 * S + 3) * DIR;
      if (js >= x.y0 && js < x.y1 && x.out_lane) {
        double2 v = s.w[S][CFD_SLOT(2 * S + 3)];
        if (RC || EDGE)
          v = open_refresh<CASE, EDGE, 3>(x, L, js, v, open_lo<DIR, ROT>(s.w[S], 2 * S + 3),
                                          open_hi<DIR, ROT>(s.w[S], 2 * S + 3));
        store_row_pair(x.pout, x.prs, (size_t)(js - x.g.row_lo) * (size_t)x.g.pitch + x.gi, v);
      }
    }
    open_sweeps<S + 1, NS, CASE, DIR, ROT, PAR, EDGE, RC>(x, L, s, R);
  }
}

constexpr int OPEN_PD = 4;  // rows of p_in / f in flight

template <int NS, int CASE, int DIR, int ROT, int PAR, bool EDGE, bool RC>
__device__ __forceinline__ void open_step(const WaveCtx<CASE>& x, const OpenLanes& L, OpenRun<NS>& s, int R) {
  constexpr int PD = OPEN_PD;
  s.w[0][CFD_SLOT(0)] = s.np[CFD_S10(0)];
  s.fr[CFD_S10(1)] = s.nf[CFD_S10(1)];
  if constexpr (!EDGE) {  // the proof's Pin: every p_in value this wave uses
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
  open_sweeps<0, NS, CASE, DIR, ROT, PAR, EDGE, RC>(x, L, s, R);
}

// one wave's band [y0, y1): dm[q] = max |black update| of sweep q over its
// proving output cells (interior-column waves; 0 on EDGE waves), pm = max |p_in|.
// RC: each group of 10 steps whose rows (the front's 10 rows, the pipeline
// behind them and their neighbours) all lie in (gmin, gmax) - no ghost row,
// no row outside the stored ones, for the step's block columns nothing at or
// above the block's lower edge - runs without row checks or row rules (RC
// false: the same instructions as an interior band), the others with them.
template <int NS, int CASE, int DIR, bool EDGE, bool RC>
__device__ __forceinline__ void open_march(const WaveCtx<CASE>& x, int y0, int y1, double (&dm)[NS], double& pm,
                                           int gmin = 0, int gmax = 0) {
  constexpr int H = 2 * NS + 1, PD = OPEN_PD;
  const int Rb0 = (DIR > 0) ? y0 - H : y1 - 1 + H;
  const int Rbeg = Rb0 - DIR * (Rb0 & 1);  // even first front row: compile-time colours
  const int nsteps = (y1 - y0) + 2 * H + (Rb0 & 1);
  const OpenLanes L = EDGE ? open_lanes(x) : OpenLanes{};
  OpenRun<NS> s;
  const double2 z = make_double2(0.0, 0.0);
#pragma unroll
  for (int k = 0; k < 5; ++k)
#pragma unroll
    for (int q = 0; q < NS; ++q) s.w[q][k] = z;
#pragma unroll
  for (int k = 0; k < 10; ++k) s.fr[k] = z;
#pragma unroll
  for (int q = 0; q < NS; ++q) s.dm[q] = 0.0;
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
  constexpr int BACK = 2 * NS + 5;  // rows behind the front a step touches (store row + neighbour + 1)
  for (int st = 0; st < nsteps; st += 10, R += 10 * DIR) {
    const int glo = (DIR > 0) ? R - BACK : R - 11, ghi = (DIR > 0) ? R + 11 : R + BACK;
    if (RC && glo > gmin && ghi < gmax) {  // (wave-uniform)
      open_step<NS, CASE, DIR, 0, 0, EDGE, false>(x, L, s, R);
      open_step<NS, CASE, DIR, 1, 1, EDGE, false>(x, L, s, R + DIR);
      open_step<NS, CASE, DIR, 2, 0, EDGE, false>(x, L, s, R + 2 * DIR);
      open_step<NS, CASE, DIR, 3, 1, EDGE, false>(x, L, s, R + 3 * DIR);
      open_step<NS, CASE, DIR, 4, 0, EDGE, false>(x, L, s, R + 4 * DIR);
      open_step<NS, CASE, DIR, 0, 1, EDGE, false>(x, L, s, R + 5 * DIR);
      open_step<NS, CASE, DIR, 1, 0, EDGE, false>(x, L, s, R + 6 * DIR);
      open_step<NS, CASE, DIR, 2, 1, EDGE, false>(x, L, s, R + 7 * DIR);
      open_step<NS, CASE, DIR, 3, 0, EDGE, false>(x, L, s, R + 8 * DIR);
      open_step<NS, CASE, DIR, 4, 1, EDGE, false>(x, L, s, R + 9 * DIR);
      continue;
    }
    open_step<NS, CASE, DIR, 0, 0, EDGE, RC>(x, L, s, R);
    open_step<NS, CASE, DIR, 1, 1, EDGE, RC>(x, L, s, R + DIR);
    open_step<NS, CASE, DIR, 2, 0, EDGE, RC>(x, L, s, R + 2 * DIR);
    open_step<NS, CASE, DIR, 3, 1, EDGE, RC>(x, L, s, R + 3 * DIR);
    open_step<NS, CASE, DIR, 4, 0, EDGE, RC>(x, L, s, R + 4 * DIR);
    open_step<NS, CASE, DIR, 0, 1, EDGE, RC>(x, L, s, R + 5 * DIR);
    open_step<NS, CASE, DIR, 1, 0, EDGE, RC>(x, L, s, R + 6 * DIR);
    open_step<NS, CASE, DIR, 2, 1, EDGE, RC>(x, L, s, R + 7 * DIR);
    open_step<NS, CASE, DIR, 3, 0, EDGE, RC>(x, L, s, R + 8 * DIR);
    open_step<NS, CASE, DIR, 4, 1, EDGE, RC>(x, L, s, R + 9 * DIR);
  }
  pm = s.pm;
#pragma unroll
  for (int q = 0; q < NS; ++q) dm[q] = (!EDGE && x.out_lane) ? s.dm[q] : 0.0;
}
#undef CFD_S10
#undef CFD_SLOT

#ifndef CFD_OPEN_MIN_WAVES
#define CFD_OPEN_MIN_WAVES 2
#endif
// diagnostic build only (CFD_OPEN_STAMPS=1, never the product library): each
// wave's march duration (shader clock) with its tile, band and path, read
// back by cfd_open_stamps (the last launch's)
#ifndef CFD_OPEN_STAMPS
#define CFD_OPEN_STAMPS 0
#endif
#if CFD_OPEN_STAMPS
constexpr int OPEN_STAMP_MAX = 8192;
__device__ long long open_stamp_buf[OPEN_STAMP_MAX * 8];
#endif

// Tiling as poisson_multi_kernel (PairPlan: boundary-column tiles in bands of
// pl.the rows, then the interior column tiles; 8-column halos, 112 output
// columns per wave).
template <int CASE, int NS>
__global__ __launch_bounds__(256, CFD_OPEN_MIN_WAVES) void poisson_open_proof_kernel(
    Geo g, Coef c, const double* __restrict__ pin, double* __restrict__ pout, const double* __restrict__ f,
    PoissonCtl ctl, int k, int ka, int kb, PairPlan pl, int flags) {
  static_assert(CASE == CHANNEL || CASE == BACKSTEP, "open cases");
  constexpr int H = 8;  // column halo
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (!(flags & 4) && !window_go_on(ctl, ka, kb, lane, blockIdx.x == 0 && wv == 0, (flags & 128) != 0)) return;
  if (blockIdx.x == 0 && wv == 0 && lane < RES_SHARDS) {
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
  const int nbe = pl.nbe0 + pl.nbe1, nbi = pl.nb0 + pl.nb1, nlb = pl.nlf + pl.nle + pl.nlt;
  const int nxb = pl.nlf + pl.nle + pl.nxt;
  int band, ctile, y0, y1;
  // band `band` of a class with bands of th rows: nb0 of them over [lo0, hi0), then [lo1, hi1)
  auto rows_of = [&](int th, int nb0) {
    const bool r0 = band < nb0;
    y0 = r0 ? pl.lo0 + band * th : pl.lo1 + (band - nb0) * th;
    y1 = min(y0 + th, r0 ? pl.hi0 : pl.hi1);
  };
  if (tile < ned * nbe) {
    const int e = tile / nbe;
    ctile = (e == 0) ? 0 : (e == 1 && ne == 2) ? pl.ctiles - 1 : (e == ne && pl.cxa > 0) ? pl.cxa - 1 : pl.cxb - 1;
    band = tile % nbe;
    rows_of(pl.the, pl.nbe0);
  } else if (tile < ned * nbe + pl.nl * nlb + pl.ncx * nxb) {  // step: the block's column tiles
    const bool left = tile < ned * nbe + pl.nl * nlb;
    const int t = left ? tile - ned * nbe : tile - ned * nbe - pl.nl * nlb;
    const int nt = left ? pl.nl : pl.ncx;
    ctile = 1 + (left ? 0 : pl.nl) + t % nt;
    band = t / nt;
    if (band < pl.nlf) {  // below the block's edge zone: interior path
      y0 = pl.lo0 + band * pl.th;
      y1 = min(y0 + pl.th, pl.lz);
    } else if (band < pl.nlf + pl.nle) {  // the edge zone
      y0 = pl.lz + (band - pl.nlf) * pl.the;
      y1 = min(y0 + pl.the, pl.le);
    } else {  // above: ghost row ny + 1 (left) / the fluid right of the block (crossing)
      y0 = (left ? pl.lt : pl.le) + (band - pl.nlf - pl.nle) * pl.the;
      y1 = min(y0 + pl.the, pl.hi0);
    }
  } else {
    const int t = tile - ned * nbe - pl.nl * nlb - pl.ncx * nxb;
    const int nci = pl.ctiles - ned - pl.nl - pl.ncx;
    if (t >= nci * nbi) return;
    ctile = 1 + pl.nl + pl.ncx + t % nci;
    band = t / nci;
    if (pl.cxa > 0 && ctile >= pl.cxa - 1) ++ctile;
    if (pl.cxb > 0 && ctile >= pl.cxb - 1) ++ctile;
    rows_of(pl.th, pl.nb0);
  }
  const int gi = ctile * PAIR_TWC - H + 2 * lane;
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
  // proving rows (interior-column waves): band rows, 2 <= j <= ny - 1
  x.py0 = max(y0, 2);
  x.py1 = min(y1, g.ny);
  const int c0 = ctile * PAIR_TWC - H;
  constexpr int CONE = 2 * NS + 2;  // rows the march reads beyond its band (pipeline + parity row)
  // interior-column wave: every column a fluid cell with fluid neighbours, off
  // the step's block: right of the block, or every row the march reads below
  // the block's lower edge row (inlet_jmax + 1, refreshed each sweep: the
  // margin mirrors `safe`'s for ghost row ny + 1)
  const bool cols_in = c0 >= 1 && c0 + 127 <= g.nx &&
                       (CASE != BACKSTEP || c0 > c.step_i + 1 || y1 + CONE < c.inlet_jmax + 1);
  if (CASE == BACKSTEP && c0 >= 1 && c0 + 127 <= c.step_i - 1 && y0 - CONE >= c.inlet_jmax + 2 &&
      y1 + CONE <= g.ny) {
    // a band inside the block, away from fluid and ghost rows / columns:
    // never updated or refreshed (both buffers hold its values)
    return;
  }
  const bool up = (flags & 1) && (band & 1);
  // interior band whose march stays in rows 1 .. ny (no ghost row, stored
  // rows only): no row checks, nothing refreshed
  const bool safe = cols_in && y0 - CONE > x.rmin && y1 + CONE < min(x.rmax, g.ny + 1);
#if CFD_OPEN_STAMPS
  long long t0_;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0_)::"memory");
#endif
  double dm[NS], pm = 0.0;
  // rows of the groups that may run without row checks: (gmin, gmax)
  const int gmin = x.rmin;
  int gmax = min(x.rmax, g.ny + 1);
  if (CASE == BACKSTEP && c0 <= c.step_i + 1) gmax = min(gmax, c.inlet_jmax);
  if (!cols_in) open_march<NS, CASE, 1, true, true>(x, y0, y1, dm, pm, gmin, gmax);
  // safe bands alternate their direction (flags bit 0) in the channel only:
  // measured neutral for the step (one copy of its loop: smaller code)
  // (the channel: 31 -> 35 us without them, profiles/r4_icache)
  else if (CASE == CHANNEL && safe && up) open_march<NS, CASE, -1, false, false>(x, y0, y1, dm, pm);
  else if (safe) open_march<NS, CASE, 1, false, false>(x, y0, y1, dm, pm);
  // (row-checked bands march down only: one copy of that code, which few
  // waves run, in the instruction cache beside the safe bands' loops; neutral
  // within noise, profiles/r4_icache)
  else open_march<NS, CASE, 1, false, true>(x, y0, y1, dm, pm, gmin, gmax);
  double growth = 1.0;
#pragma unroll
  for (int q = 0; q < NS; ++q) growth *= 9.0;
  const double pinv = wave_max(pm), F = ctl.tol[2], tol = ctl.tol[0];
  double r[NS];
#pragma unroll
  for (int q = 0; q < NS; ++q) r[q] = proof_ratio_gen(c, tol, wave_max(dm[q]), pinv, F, growth);
#if CFD_OPEN_STAMPS
  {
    long long t1_;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1_)::"memory");
    if (tile < OPEN_STAMP_MAX && lane < 8) {
      const long long v[8] = {tile, ctile, band, y0, y1, cols_in ? 1 : 0, safe ? 1 : 0, t1_ - t0_};
      long long o = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) o = lane == q ? v[q] : o;
      open_stamp_buf[(size_t)tile * 8 + lane] = o;
    }
  }
#endif
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      double* sl = ctl.ring + (size_t)((k + q) & (RING - 1)) * RES_SHARDS * SHARD_STRIDE;
      atomicMax(reinterpret_cast<unsigned long long*>(sl + (size_t)(tile % RES_SHARDS) * SHARD_STRIDE),
                (unsigned long long)__double_as_longlong(r[q]));
    }
  }
}

#if CFD_OPEN_STAMPS
// diagnostic build only: per wave {tile, column tile, band, y0, y1, interior
// columns, safe, cycles} of the last open proof launch
extern "C" int cfd_open_stamps(long long* out, int n) {
  if (n > OPEN_STAMP_MAX * 8) n = OPEN_STAMP_MAX * 8;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(open_stamp_buf), (size_t)n * 8) == hipSuccess ? n : -1;
}
#endif

void open_proof_launch(int case_id, int ns, const Geo& g, const Coef& c, const double* pin, double* pout,
                       const double* f, const PoissonCtl& ctl, int k, int ka, int kb, const PairPlan& pl, int flags,
                       hipStream_t st) {
  const int ntiles = plan_waves(pl);
  if (ntiles == 0) return;
  const dim3 grid((ntiles + 3) / 4);
#define CFD_OPEN_LAUNCH(CASE, NS) \
  poisson_open_proof_kernel<CASE, NS><<<grid, 256, 0, st>>>(g, c, pin, pout, f, ctl, k, ka, kb, pl, flags)
  if (case_id == CHANNEL) {
    if (ns == 4) CFD_OPEN_LAUNCH(CHANNEL, 4); else CFD_OPEN_LAUNCH(CHANNEL, 3);
  } else {
    if (ns == 4) CFD_OPEN_LAUNCH(BACKSTEP, 4); else CFD_OPEN_LAUNCH(BACKSTEP, 3);
  }
#undef CFD_OPEN_LAUNCH
}

}  // namespace cfd
