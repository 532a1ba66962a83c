// smlex.hip — the reference's own (lexicographic) SOR order on a
// reference-sized grid: the whole solve in one workgroup, p in LDS, bit for
// bit the reference's loop (cavity-01.cpp:633-678, channel-01.cpp:652-682,
// backwards_step-01.cpp:893-931).
//
// The reference's runs (cavity 63², channel 93×31, step 256×32) are launch
// bound in the multi-block reference-order march (lexw.hpp: 13-22 µs per
// iteration); here one 16-wave workgroup runs every iteration
// with one barrier per half-sweep.
//
// Schedule. With a 5-point stencil the Gauss-Seidel sweep in j-then-i order is
// a red-black half-sweep sequence with a time skew: cell (j,i), d = i + j,
// performs its iteration k at half-sweep H = d - 2 + 2(k-1), reading W and S
// at iteration k (updated at H-1) and E, N and itself at k-1 (E, N update
// next at H+1). So one array P updated in place, half-sweep by half-sweep, is
// exactly the reference's sweep. Ghosts and the step's solid cells take the
// refresh that follows each sweep (channel-01.cpp:531-540,
// backwards_step-01.cpp:685-738) from their only fluid neighbour, which writes
// them right after its update: ghost = its value (outlet: 0), solid =
// (0 + value) / 1. The step's block corner averages two fluid cells, A below
// it and B to its right (((0 + B) + A) / 2), which update in the same
// half-sweep (A at iteration k, B at k-1): one thread owns both and runs B,
// the corner, then A.
//
// Residuals. The residual of iteration k of cell c needs its W, S at
// iteration k, which update again in the half-sweep after c's: every update
// also keeps the cell's previous value in Q, so c evaluates its iteration-(k-1)
// residual while performing iteration k (P: itself, E, N, ghosts, solids;
// Q: interior W, S). Only "some cell of iteration k exceeds tol" matters for
// the stop rule, so each cell sets flag[k] (a plain store; the ring of
// SMLEX_NF iterations in flight); iteration k is complete after the last cell
// (d = nx + ny) ran iteration k + 1, tested by every thread after that
// half-sweep's barrier. A stop at k finds cells near (1,1) up to (nx+ny)/2
// iterations further: the solve then restores the last checkpoint before k
// (every cell stores its value at iterations that are multiples of M into one
// of SMLEX_NCK global buffers, so the one needed is never overwritten) or the
// initial field, and replays to exactly k with no tests. The reported
// residual is the final field's (the same formula and operands as the
// reference's last evaluation). The last iteration's write-backs are skipped,
// so ghosts and solids then hold the refresh after iteration K-1 as the
// reference's final refresh reads them; the tail applies that refresh.
//
// LDS: P and Q ((nx+2)(ny+2) doubles each, at most SMLEX_CELLS) + the flag
// ring. Cells of each colour are numbered row by row and dealt to the 1024
// threads once (their (j,i), source value and refresh duties stay in
// registers), as in small.hpp.
#include "smlex.hpp"

#include <algorithm>

namespace cfd {

namespace {

constexpr int KQW = 1, KQS = 2;                  // residual reads Q for the W / S neighbour (interior fluid)
constexpr int KGW = 4, KGS = 8, KGN = 16, KGE = 32;  // writes ghost (j,0) / (0,i) / (ny+1,i) / (j,nx+1) = 0
constexpr int KSN = 64, KSW = 128;               // step: writes the solid above / left of it ((0 + v) / 1)
constexpr int KE = 256, KW = 512, KN = 1024;     // cavity indicators eps_e, eps_w, eps_n (cavity-01.cpp:640-643)

template <int CASE>
__device__ __forceinline__ int cell_kind(const Coef& c, int nx, int ny, int j, int i) {
  int k = 0;
  if (is_fluid(c, nx, ny, j, i - 1)) k |= KQW;
  if (is_fluid(c, nx, ny, j - 1, i)) k |= KQS;
  if (CASE == CAVITY) {
    if (i < nx) k |= KE;
    if (i > 1) k |= KW;
    if (j < ny) k |= KN;
  } else {
    if (i == 1) k |= KGW;
    if (j == 1) k |= KGS;
    if (j == ny) k |= KGN;
    if (i == nx) k |= KGE;
  }
  if (CASE == BACKSTEP) {
    if (j == c.inlet_jmax && i < c.step_i) k |= KSN;
    if (i == c.step_i + 1 && j > c.inlet_jmax + 1) k |= KSW;
  }
  return k;
}

// The cavity's indicators as multipliers (1.0 / 0.0; for finite x, 0.0 * x ==
// the reference's int 0 * x and 1.0 * x == x) and omega / neighbour_count:
// the update and the residual become straight-line (small.hpp PRE)
struct CavMul {
  double me, mw, mn, om;
};
__device__ __forceinline__ CavMul cav_mul(const Coef& c, int kind) {
  const int n = ((kind & KE) ? 1 : 0) + ((kind & KW) ? 1 : 0) + ((kind & KN) ? 1 : 0) + 1;
  double o1 = c.om_nc[1], o2 = c.om_nc[2], o3 = c.om_nc[3], o4 = c.om_nc[4];
  asm("" : "+s"(o1), "+s"(o2), "+s"(o3), "+s"(o4));  // (values, not an index into Coef: device.hpp sor_update)
  return {(kind & KE) ? 1.0 : 0.0, (kind & KW) ? 1.0 : 0.0, (kind & KN) ? 1.0 : 0.0,
          n == 4 ? o4 : n == 3 ? o3 : n == 2 ? o2 : o1};
}

// One cell's operands in a half-sweep (loaded before any of the thread's
// cells is stored: the cells of one colour never read each other)
struct Ops {
  double pc, pE, pN, pW, pS, rW, rS;
};
__device__ __forceinline__ Ops cell_load(const double* P, const double* Q, int W, int o, int kind) {
  Ops x;
  x.pc = P[o];
  x.pE = P[o + 1];
  x.pN = P[o + W];
  x.pW = P[o - 1];
  x.pS = P[o - W];
  // iteration k-1 of this cell's W, S (they moved on to k): Q for interior
  // fluid cells, P for ghosts and solids (refreshed from this cell)
  x.rW = (kind & KQW) ? Q[o - 1] : x.pW;
  x.rS = (kind & KQS) ? Q[o - W] : x.pS;
  return x;
}

// The update to iteration k and, when tested, whether the cell's residual of
// iteration k-1 exceeds tol (cavity-01.cpp:643-677, channel-01.cpp:659-681)
template <int CASE>
__device__ __forceinline__ double cell_compute(const Coef& c, const Ops& x, const CavMul& m, double fq, bool test,
                                               double tol, bool& exceeds) {
  if (CASE == CAVITY) {
    if (test) {
      const double r = c.idx2 * (((m.me * (x.pE - x.pc) + m.mw * (x.rW - x.pc)) + m.mn * (x.pN - x.pc)) +
                                 (x.rS - x.pc)) - fq;
      exceeds = fabs(r) > tol;
    }
    return x.pc * c.one_m_omega + m.om * ((x.pE * m.me + x.pW * m.mw) + (x.pN * m.mn + x.pS) - fq * c.h2);
  } else {
    if (test) {
      const double lap = (x.pE - 2.0 * x.pc + x.rW) * c.idx2 + (x.pN - 2.0 * x.pc + x.rS) * c.idy2;
      exceeds = fabs(lap - fq) > tol;
    }
    return sor_interior<CASE>(c, x.pc, x.pW, x.pE, x.pS, x.pN, fq);
  }
}

// Stores of one cell: the new value, its previous value (Q), the ghosts /
// solids it feeds (not after the solve's last iteration kcap), the flag of
// its iteration k-1, the checkpoint (iterations k = multiples of 2^mlog)
template <int CASE>
__device__ __forceinline__ void cell_store(double* P, double* Q, int* flag, double* ck, int ncell, int W, int o,
                                           int kind, double pc, double nv, int k, int kcap, bool exceeds, int mlog) {
  P[o] = nv;
  Q[o] = pc;
  if (exceeds) flag[(k - 1) & (SMLEX_NF - 1)] = 1;
  if (CASE != CAVITY && k < kcap) {
    if (kind & KGW) P[o - 1] = nv;
    if (kind & KGS) P[o - W] = nv;
    if (kind & KGN) P[o + W] = nv;
    if (kind & KGE) P[o + 1] = 0.0;
    if (CASE == BACKSTEP) {
      if (kind & KSN) P[o + W] = (0.0 + nv) / 1;
      if (kind & KSW) P[o - 1] = (0.0 + nv) / 1;
    }
  }
  if (mlog >= 0 && (k & ((1 << mlog) - 1)) == 0) ck[(size_t)((k >> mlog) & (SMLEX_NCK - 1)) * ncell + o] = nv;
}

// One whole cell (the special thread's sequence B, corner, A)
template <int CASE>
__device__ __forceinline__ double cell_step(const Coef& c, double* P, double* Q, int* flag, double* ck, int ncell,
                                            int W, int j, int i, int kind, double fq, int k, bool test, int kcap,
                                            int mlog, double tol) {
  const int o = j * W + i;
  const Ops x = cell_load(P, Q, W, o, kind);
  bool ex = false;
  const double nv = cell_compute<CASE>(c, x, cav_mul(c, kind), fq, test, tol, ex);
  cell_store<CASE>(P, Q, flag, ck, ncell, W, o, kind, x.pc, nv, k, kcap, ex, mlog);
  return nv;
}

// ghosts (channel-01.cpp:531-540, backwards_step-01.cpp:685-703) from the
// current interior, then the step's solids next to fluid (:706-738)
template <int CASE>
__device__ void refresh_all(const Coef& c, int nx, int ny, int W, double* P) {
  if (CASE == CAVITY) return;
  const int t = threadIdx.x;
  for (int e = t; e < ny + nx; e += SMLEX_THREADS) {
    if (e < ny) {
      const int j = e + 1;
      P[j * W] = P[j * W + 1];
      P[j * W + nx + 1] = 0.0;
    } else {
      const int i = e - ny + 1;
      P[i] = P[W + i];
      P[(ny + 1) * W + i] = P[ny * W + i];
    }
  }
  __syncthreads();
  if (CASE == BACKSTEP) {
    for (int e = t; e < nx * ny; e += SMLEX_THREADS) {
      const int j = 1 + e / nx, i = 1 + e % nx;
      if (is_fluid(c, nx, ny, j, i)) continue;
      const int o = j * W + i;
      double out;
      if (refresh_value<CASE>(c, nx, ny, j, i, P[o], P[o - 1], P[o + 1], P[o - W], P[o + W], out)) P[o] = out;
    }
    __syncthreads();
  }
}

template <int CASE, int MAXC>
__global__ __launch_bounds__(SMLEX_THREADS) void poisson_smlex_kernel(Geo g, Coef c, double* __restrict__ p,
                                                                      const double* __restrict__ f,
                                                                      const double* __restrict__ tolv, int max_iters,
                                                                      double* __restrict__ ck, int mlog,
                                                                      int* __restrict__ out_iters,
                                                                      double* __restrict__ out_res) {
  __shared__ double P[SMLEX_CELLS];
  __shared__ double Q[SMLEX_CELLS];
  __shared__ int flag[SMLEX_NF];
  __shared__ unsigned long long s_res;
  const int t = threadIdx.x, lane = t & 63;
  const int nx = g.nx, ny = g.ny, W = nx + 2, ncell = W * (ny + 2);
  const int dmax = nx + ny;  // the last cell (ny, nx) is fluid in every case
  auto gidx = [&](int j, int i) { return (size_t)(j - g.row_lo) * (size_t)g.pitch + (size_t)i; };
  const double tol = tolv[0];
  if (!(tolv[1] > tol) || max_iters <= 0) {  // the loop is never entered (cavity-01.cpp:633)
    if (t == 0) {
      *out_iters = 0;
      *out_res = tolv[1];
    }
    return;
  }
  for (int e = t; e < ncell; e += SMLEX_THREADS) {
    const int j = e / W, i = e - j * W;
    P[e] = p[gidx(j, i)];
  }
  for (int e = t; e < SMLEX_NF; e += SMLEX_THREADS) flag[e] = 0;
  if (t == 0) s_res = 0ull;

  // this thread's cells of each colour (i + j even: colour 0), numbered row
  // by row like small.hpp; the step's A and B go to the special thread
  const int jc = c.inlet_jmax + 1, ic = c.step_i;  // the step's block corner (solid)
  // the cavity's indicator multipliers stay in registers while they fit
  // (small.hpp PRE: up to 2 cells per thread and colour)
  constexpr bool PRE = CASE == CAVITY && MAXC <= 2;
  int cell[2][MAXC], kind[2][MAXC];
  double fc[2][MAXC];
  CavMul cm[2][PRE ? MAXC : 1];
#pragma unroll
  for (int col = 0; col < 2; ++col) {
#pragma unroll
    for (int q = 0; q < MAXC; ++q) {
      const int e = t + q * SMLEX_THREADS;
      int v = -1, kd = 0;
      double fv = 0.0;
      const int pr = e / nx, r = e - pr * nx;  // two rows hold nx cells of each colour
      int j = 1 + 2 * pr;
      const int i0 = 1 + ((j + 1 + col) & 1);
      const int n1 = (nx - i0) / 2 + 1;
      int i;
      if (r < n1) {
        i = i0 + 2 * r;
      } else {
        ++j;
        i = 1 + ((j + 1 + col) & 1) + 2 * (r - n1);
      }
      const bool spec = CASE == BACKSTEP && ((j == jc - 1 && i == ic) || (j == jc && i == ic + 1));
      if (j <= ny && i <= nx && is_fluid(c, nx, ny, j, i) && !spec) {
        v = (j << 16) | i;
        kd = cell_kind<CASE>(c, nx, ny, j, i);
        fv = f[gidx(j, i)];
      }
      cell[col][q] = v;
      kind[col][q] = kd;
      fc[col][q] = fv;
      if constexpr (PRE) cm[col][PRE ? q : 0] = cav_mul(c, kd);
    }
  }
  // the special thread: B = (jc, ic+1), then the corner, then A = (jc-1, ic)
  const bool spt = CASE == BACKSTEP && t == SMLEX_THREADS - 1;
  const int colAB = (jc - 1 + ic) & 1;
  int kindA = 0, kindB = 0;
  double fA = 0.0, fB = 0.0;
  if (spt) {
    kindA = cell_kind<CASE>(c, nx, ny, jc - 1, ic);
    kindB = cell_kind<CASE>(c, nx, ny, jc, ic + 1);
    fA = f[gidx(jc - 1, ic)];
    fB = f[gidx(jc, ic + 1)];
  }
  __syncthreads();

  int kbase = 0, kcap = max_iters, K = -1;
  bool replay = false;
  int Hend = dmax - 2 + 2 * (kcap - 1);  // the last cell's last update
  for (int H = 0;; ++H) {
    const int col = H & 1;
    const int ml = replay ? -1 : mlog;
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      if (cc != col) continue;
      // groups of (up to) two cells: every operand of the group first (the
      // cells of one colour never read each other: the loads of both in
      // flight together), then the arithmetic, then the stores
      constexpr int G = 2;
#pragma unroll
      for (int q0 = 0; q0 < MAXC; q0 += G) {
        constexpr int GN = G;
        Ops x[GN];
        int kq[GN], oq[GN];
        bool act[GN];
#pragma unroll
        for (int u = 0; u < GN; ++u) {
          const int q = q0 + u < MAXC ? q0 + u : MAXC - 1;
          const int v = (q0 + u < MAXC) ? cell[cc][q] : -1;
          const int j = v >> 16, i = v & 0xffff;
          kq[u] = kbase + ((H - (i + j) + 2) >> 1) + 1;
          act[u] = v >= 0 && kq[u] > kbase && kq[u] <= kcap;
          oq[u] = act[u] ? j * W + i : W + 1;  // (an inactive slot loads a harmless cell)
          x[u] = cell_load(P, Q, W, oq[u], kind[cc][q]);
        }
        double nv[GN];
        bool ex[GN];
#pragma unroll
        for (int u = 0; u < GN; ++u) {
          const int q = q0 + u < MAXC ? q0 + u : MAXC - 1;
          ex[u] = false;
          const CavMul m = PRE ? cm[cc][PRE ? q : 0] : cav_mul(c, kind[cc][q]);
          nv[u] = cell_compute<CASE>(c, x[u], m, fc[cc][q], !replay && kq[u] >= 2, tol, ex[u]);
        }
#pragma unroll
        for (int u = 0; u < GN; ++u) {
          const int q = q0 + u < MAXC ? q0 + u : MAXC - 1;
          if (act[u])
            cell_store<CASE>(P, Q, flag, ck, ncell, W, oq[u], kind[cc][q], x[u].pc, nv[u], kq[u], kcap, ex[u], ml);
        }
      }
    }
    if (spt && col == colAB) {
      const int kB = kbase + ((H - (jc + ic + 1) + 2) >> 1) + 1, kA = kB + 1;
      if (kB > kbase && kB <= kcap) {
        const double b = cell_step<CASE>(c, P, Q, flag, ck, ncell, W, jc, ic + 1, kindB, fB, kB,
                                         !replay && kB >= 2, kcap, ml, tol);
        if (kB < kcap) P[jc * W + ic] = ((0.0 + b) + P[(jc - 1) * W + ic]) / 2;  // A at iteration kB
      }
      if (kA > kbase && kA <= kcap)
        cell_step<CASE>(c, P, Q, flag, ck, ncell, W, jc - 1, ic, kindA, fA, kA, !replay && kA >= 2, kcap, ml, tol);
    }
    __syncthreads();
    // decisions (every thread the same)
    if (replay) {
      if (H >= Hend) break;
      continue;
    }
    if (H >= dmax && ((H - dmax) & 1) == 0) {  // iteration kc complete: the reference's while test
      const int kc = ((H - dmax) >> 1) + 1;
      if (t == 0 && kc >= 2) flag[(kc - 1) & (SMLEX_NF - 1)] = 0;  // (read by every thread at the last test)
      if (kc < max_iters && flag[kc & (SMLEX_NF - 1)] == 0) K = kc;
    }
    if (K < 0) {
      if (H >= Hend) {  // the cap: every cell ran max_iters iterations
        K = max_iters;
        break;
      }
      continue;
    }
    // converged at K < max_iters: restore the last checkpoint before K (or the
    // initial field) and replay to exactly K
    const int mstar = ((K - 1) >> mlog) << mlog;
    __threadfence();  // (the checkpoint stores of every wave, then read back by others)
    __syncthreads();
    __threadfence();
    if (mstar == 0) {
      for (int e = t; e < ncell; e += SMLEX_THREADS) {
        const int j = e / W, i = e - j * W;
        P[e] = p[gidx(j, i)];
      }
      __syncthreads();
    } else {
      const double* src = ck + (size_t)((mstar >> mlog) & (SMLEX_NCK - 1)) * ncell;
      for (int e = t; e < ncell; e += SMLEX_THREADS) {
        const int j = e / W, i = e - j * W;
        if (is_fluid(c, nx, ny, j, i)) P[e] = src[e];
      }
      __syncthreads();
      refresh_all<CASE>(c, nx, ny, W, P);  // the field after iteration mstar's refresh
    }
    kbase = mstar;
    kcap = K;
    replay = true;
    Hend = dmax - 2 + 2 * (kcap - kbase - 1);
    H = -1;
  }

  // the final refresh (the reference's last applyPressureGhosts): ghosts from
  // the final interior with the solids as refreshed after iteration K-1, then
  // the solids
  refresh_all<CASE>(c, nx, ny, W, P);
  // the reported residual: max-norm of the final field (cavity-01.cpp:659-677)
  double m = 0.0;
#pragma unroll
  for (int cc = 0; cc < 2; ++cc)
#pragma unroll
    for (int q = 0; q < MAXC; ++q) {
      const int v = cell[cc][q];
      if (v < 0) continue;
      const int j = v >> 16, i = v & 0xffff, o = j * W + i;
      m = fmax(m, residual_abs<CASE>(c, nx, ny, j, i, P[o], P[o - 1], P[o + 1], P[o - W], P[o + W], fc[cc][q]));
    }
  if (spt) {
    int o = (jc - 1) * W + ic;
    m = fmax(m, residual_abs<CASE>(c, nx, ny, jc - 1, ic, P[o], P[o - 1], P[o + 1], P[o - W], P[o + W], fA));
    o = jc * W + ic + 1;
    m = fmax(m, residual_abs<CASE>(c, nx, ny, jc, ic + 1, P[o], P[o - 1], P[o + 1], P[o - W], P[o + W], fB));
  }
  m = wave_max(m);
  if (lane == 0) atomicMax(&s_res, (unsigned long long)__double_as_longlong(m));
  __syncthreads();
  if (t == 0) {
    *out_iters = K;
    *out_res = __longlong_as_double((long long)s_res);
  }
  for (int e = t; e < ncell; e += SMLEX_THREADS) {
    const int j = e / W, i = e - j * W;
    p[gidx(j, i)] = P[e];
  }
}

}  // namespace

bool smlex_fits(const Geo& g, const Coef& c) {
  const long long cells = (long long)(g.nx + 2) * (g.ny + 2);
  if (cells > SMLEX_CELLS || (g.nx + g.ny) / 2 + 8 >= SMLEX_NF) return false;
  if (g.nx > 0xffff || g.ny > 0x7fff) return false;
  if (c.case_id == BACKSTEP) {  // a corner cell with fluid below and to the right
    if (!(c.step_i >= 2 && c.step_i <= g.nx - 1 && c.inlet_jmax >= 1 && c.inlet_jmax <= g.ny - 2)) return false;
  }
  return true;
}

int smlex_interval(int nx, int ny) {
  int m = 8;
  while (m < (nx + ny) / 6 + 2) m *= 2;  // (a power of two: iterations test it with a mask)
  return m;
}

void smlex_launch(int case_id, const Geo& g, const Coef& c, double* p, const double* f, const double* tolv,
                  int max_iters, double* ck, int* out_iters, double* out_res, hipStream_t st) {
  const long long per_colour = ((long long)g.nx * g.ny + 1) / 2;
  const int maxc = per_colour <= 2 * SMLEX_THREADS ? 2 : per_colour <= 4 * SMLEX_THREADS ? 4 : 5;
  int mlog = 0;
  while ((1 << mlog) < smlex_interval(g.nx, g.ny)) ++mlog;
#define CFD_SMLEX(CASE)                                                                                         \
  if (maxc == 2)                                                                                                \
    poisson_smlex_kernel<CASE, 2><<<1, SMLEX_THREADS, 0, st>>>(g, c, p, f, tolv, max_iters, ck, mlog, out_iters, out_res); \
  else if (maxc == 4)                                                                                           \
    poisson_smlex_kernel<CASE, 4><<<1, SMLEX_THREADS, 0, st>>>(g, c, p, f, tolv, max_iters, ck, mlog, out_iters, out_res); \
  else                                                                                                          \
    poisson_smlex_kernel<CASE, 5><<<1, SMLEX_THREADS, 0, st>>>(g, c, p, f, tolv, max_iters, ck, mlog, out_iters, out_res)
  if (case_id == CAVITY) { CFD_SMLEX(CAVITY); }
  else if (case_id == CHANNEL) { CFD_SMLEX(CHANNEL); }
  else { CFD_SMLEX(BACKSTEP); }
#undef CFD_SMLEX
}

}  // namespace cfd
