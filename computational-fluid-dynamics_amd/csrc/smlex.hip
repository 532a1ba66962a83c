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
// Residuals. The residual of iteration k of cell c needs c, W, S, E, N at
// iteration k. c performs iteration k+1 two half-sweeps after iteration k, from
// E(k) and N(k) (the same loads serve both) while W and S have moved on to
// k+1 - but W(k) and S(k) are exactly the fresh W, S values its iteration-k
// update read: each thread keeps them (and its cells' own values) in
// registers, so c evaluates its iteration-k residual with its iteration-(k+1)
// update, from four LDS loads. (Ghost and solid W / S: the loaded value, the
// refresh after iteration k, serves both.) Only "some cell of iteration k
// exceeds tol" matters for the stop rule, so each cell sets flag[k] (a plain
// store; a ring of SMLEX_NF iterations in flight); iteration k is complete
// after the last cell (d = nx + ny) ran iteration k + 1, tested by every thread
// after that half-sweep's barrier. A stop at k finds cells near (1,1) up to
// (nx+ny)/2 iterations further: the solve then restores the last checkpoint
// before k (every cell stores its value at iterations that are multiples of
// M = 2^mlog into one of SMLEX_NCK global buffers, so the one needed is never
// overwritten) or the initial field, and replays to exactly k with no tests.
// The reported residual is the final field's (the same formula and operands
// as the reference's last evaluation). The last iteration's write-backs are
// skipped, so ghosts and solids then hold the refresh after iteration K-1 as
// the reference's final refresh reads them; the tail applies that refresh.
//
// LDS: p and the source (2 x ~(nx+2)(ny+2) doubles in a colour-split layout,
// at most SMLEX_CELLS together) + the flag ring. Cells of
// each colour are numbered row by row and dealt to the 1024 threads once
// (their (j,i), saved W / S values and refresh
// duties stay in registers), as in small.hpp.
#include "smlex.hpp"

#include <algorithm>

namespace cfd {

namespace {

constexpr int KQW = 1, KQS = 2;                  // residual takes the saved W / S value (interior fluid neighbour)
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

// A cell's register state: W / S as its last update read them
struct Own {
  double sw, ss, pc;  // (pc: its own value, kept while the registers allow: MAXC <= 2)
};

// LDS layout: row-major, (nx+2) doubles per row (the reference's (j, i)).
struct Lay {
  int w;  // doubles per row
  __device__ __forceinline__ int at(int j, int i) const { return j * w + i; }
};
struct Nb {
  int o, w, e, n, s;
};
__device__ __forceinline__ Nb nbrs_o(const Lay& L, int o) { return {o, o - 1, o + 1, o + L.w, o - L.w}; }
__device__ __forceinline__ Nb nbrs(const Lay& L, int j, int i) { return nbrs_o(L, L.at(j, i)); }

// The update of a cell to iteration k from its neighbours' loaded values and
// its own, and when tested whether its residual of iteration k-1 exceeds tol
// (cavity-01.cpp:643-677, channel-01.cpp:659-681)
template <int CASE>
__device__ __forceinline__ double cell_compute(const Coef& c, const Own& s, int kind, double pc, double pE, double pN,
                                               double pW, double pS, const CavMul& m, double fq, bool test,
                                               double tol, bool& exceeds) {
  const double rW = (kind & KQW) ? s.sw : pW;
  const double rS = (kind & KQS) ? s.ss : pS;
  if (CASE == CAVITY) {
    if (test) {
      const double r = c.idx2 * (((m.me * (pE - pc) + m.mw * (rW - pc)) + m.mn * (pN - pc)) + (rS - pc)) - fq;
      exceeds = fabs(r) > tol;
    }
    return pc * c.one_m_omega + m.om * ((pE * m.me + pW * m.mw) + (pN * m.mn + pS) - fq * c.h2);
  } else {
    if (test) {
      const double lap = (pE - 2.0 * pc + rW) * c.idx2 + (pN - 2.0 * pc + rS) * c.idy2;
      exceeds = fabs(lap - fq) > tol;
    }
    return sor_interior<CASE>(c, pc, pW, pE, pS, pN, fq);
  }
}

// Stores of one cell: the new value, the ghosts / solids it feeds (not after
// the solve's last iteration kcap), the flag of its iteration k-1, the
// checkpoint (iterations k = multiples of 2^mlog; mlog < 0: none)
template <int CASE>
__device__ __forceinline__ void cell_store(double* P, int* flag, double* ck, int ncell, const Nb& b, int kind,
                                           double nv, int k, int kcap, bool exceeds, int mlog) {
  P[b.o] = nv;
  if (exceeds) flag[(k - 1) & (SMLEX_NF - 1)] = 1;
  if (CASE != CAVITY && (kind & (KGW | KGS | KGN | KGE | KSN | KSW)) && k < kcap) {
    if (kind & KGW) P[b.w] = nv;
    if (kind & KGS) P[b.s] = nv;
    if (kind & KGN) P[b.n] = nv;
    if (kind & KGE) P[b.e] = 0.0;
    if (CASE == BACKSTEP) {
      if (kind & KSN) P[b.n] = (0.0 + nv) / 1;
      if (kind & KSW) P[b.w] = (0.0 + nv) / 1;
    }
  }
  if (mlog >= 0 && (k & ((1 << mlog) - 1)) == 0) ck[(size_t)((k >> mlog) & (SMLEX_NCK - 1)) * ncell + b.o] = nv;
}

// One whole cell (the special thread's sequence B, corner, A)
template <int CASE>
__device__ __forceinline__ double cell_step(const Coef& c, double* P, int* flag, double* ck, int ncell, const Nb& b,
                                            int kind, double fq, Own& s, int k, bool test, int kcap, int mlog,
                                            double tol) {
  const double pc = P[b.o], pE = P[b.e], pN = P[b.n], pW = P[b.w], pS = P[b.s];
  bool ex = false;
  const double nv = cell_compute<CASE>(c, s, kind, pc, pE, pN, pW, pS, cav_mul(c, kind), fq, test, tol, ex);
  cell_store<CASE>(P, flag, ck, ncell, b, kind, nv, k, kcap, ex, mlog);
  s = {pW, pS, nv};
  return nv;
}

// ghosts (channel-01.cpp:531-540, backwards_step-01.cpp:685-703) from the
// current interior, then the step's solids next to fluid (:706-738)
template <int CASE>
__device__ void refresh_all(const Coef& c, int nx, int ny, const Lay& L, double* P) {
  if (CASE == CAVITY) return;
  const int t = threadIdx.x;
  for (int e = t; e < ny + nx; e += SMLEX_THREADS) {
    if (e < ny) {
      const int j = e + 1;
      P[L.at(j, 0)] = P[L.at(j, 1)];
      P[L.at(j, nx + 1)] = 0.0;
    } else {
      const int i = e - ny + 1;
      P[L.at(0, i)] = P[L.at(1, i)];
      P[L.at(ny + 1, i)] = P[L.at(ny, i)];
    }
  }
  __syncthreads();
  if (CASE == BACKSTEP) {
    for (int e = t; e < nx * ny; e += SMLEX_THREADS) {
      const int j = 1 + e / nx, i = 1 + e % nx;
      if (is_fluid(c, nx, ny, j, i)) continue;
      const Nb b = nbrs(L, j, i);
      double out;
      if (refresh_value<CASE>(c, nx, ny, j, i, P[b.o], P[b.w], P[b.e], P[b.s], P[b.n], out)) P[b.o] = out;
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
  __shared__ int flag[SMLEX_NF];
  __shared__ unsigned long long s_res;
  const int t = threadIdx.x, lane = t & 63;
  const int nx = g.nx, ny = g.ny, W = nx + 2;
  const Lay L{W};
  const int ncell = W * (ny + 2);  // (LDS doubles of p; checkpoints use the same indices)
  // more than 2 cells per thread and colour: the source in LDS too (F, after p;
  // smlex_fits), else in registers
  constexpr bool FLDS = MAXC > 2;
  double* F = P + ncell;
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
    if (FLDS) F[e] = f[gidx(j, i)];
  }
  for (int e = t; e < SMLEX_NF; e += SMLEX_THREADS) flag[e] = 0;
  if (t == 0) s_res = 0ull;

  // this thread's cells of each colour (i + j even: colour 0), numbered row
  // by row like small.hpp; the step's A and B go to the special thread. Per
  // cell: co = kind << 15 | o (o = its LDS index < 2^15; -1: none) and kof,
  // with its iteration at half-sweep H = kbase + (H >> 1) + 2 + kof
  const int jc = c.inlet_jmax + 1, ic = c.step_i;  // the step's block corner (solid)
  // the cavity's multipliers per cell stay in registers while they fit (up to
  // 2 cells per thread and colour; else from the kind bits at each update)
  constexpr bool PRE = CASE == CAVITY && MAXC <= 2;
  constexpr bool PCREG = MAXC <= 2;  // the cells' own values in registers
  int co[2][MAXC], kof[2][MAXC];
  double fc[2][FLDS ? 1 : MAXC];
  Own own[2][MAXC];
  CavMul cm[2][PRE ? MAXC : 1];  // (PRE: the whole multiplier set per cell, small.hpp's PRE)
#pragma unroll
  for (int col = 0; col < 2; ++col) {
#pragma unroll
    for (int q = 0; q < MAXC; ++q) {
      const int e = t + q * SMLEX_THREADS;
      int v = -1, kd = 0, ko = 0;
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
        kd = cell_kind<CASE>(c, nx, ny, j, i);
        v = (kd << 15) | L.at(j, i);
        ko = -((i + j) >> 1);
        fv = f[gidx(j, i)];
      }
      co[col][q] = v;
      kof[col][q] = ko;
      if constexpr (!FLDS) fc[col][FLDS ? 0 : q] = fv;
      own[col][q] = {0.0, 0.0, 0.0};
      if constexpr (PRE) cm[col][PRE ? q : 0] = cav_mul(c, kd);
    }
  }
  // the special thread: B = (jc, ic+1), then the corner, then A = (jc-1, ic)
  const bool spt = CASE == BACKSTEP && t == SMLEX_THREADS - 1;
  const int colAB = (jc - 1 + ic) & 1;
  const Nb bA = nbrs(L, jc - 1, ic), bB = nbrs(L, jc, ic + 1);
  const int oC = L.at(jc, ic);
  int kindA = 0, kindB = 0;
  double fA = 0.0, fB = 0.0;
  __shared__ Own s_own[2];  // the special thread's A, B (in LDS: every lane would hold them in registers)
  Own& ownA = s_own[0];
  Own& ownB = s_own[1];
  if (spt) {
    kindA = cell_kind<CASE>(c, nx, ny, jc - 1, ic);
    kindB = cell_kind<CASE>(c, nx, ny, jc, ic + 1);
    fA = f[gidx(jc - 1, ic)];
    fB = f[gidx(jc, ic + 1)];
  }
  __syncthreads();
  auto load_own = [&]() {  // (own values from P: at the start and after a restore)
    if constexpr (PCREG) {
#pragma unroll
      for (int col = 0; col < 2; ++col)
#pragma unroll
        for (int q = 0; q < MAXC; ++q)
          if (co[col][q] >= 0) own[col][q].pc = P[co[col][q] & 0x7fff];
    }
  };
  load_own();

  int kbase = 0, kcap = max_iters, K = -1;
  bool replay = false;
  int Hend = dmax - 2 + 2 * (kcap - 1);  // the last cell's last update
  // the reference's while test of iteration kc is due once the barrier after
  // half-sweep dmax - 2 + 2 kc has passed; it is read during the next
  // half-sweep (its LDS load in flight with the cells' loads) and decided
  // after that one's barrier (pend: the iteration whose flag is being read)
  int pend = 0;
  for (int H = 0;; ++H) {
    const int col = H & 1;
    const int ml = replay ? -1 : mlog;
    const int fl = pend > 0 ? __builtin_amdgcn_readfirstlane(flag[pend & (SMLEX_NF - 1)]) : 1;
    const int hk = kbase + (H >> 1) + 2;  // a cell's iteration: hk + kof
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      if (cc != col) continue;
      // groups of (up to) two cells: the neighbours of both first (the cells
      // of one colour never read each other: the loads of both in flight
      // together), then the arithmetic, then the stores
      constexpr int G = (CASE == CAVITY || (CASE == BACKSTEP && MAXC >= 4)) ? 1 : 2;
#pragma unroll
      for (int q0 = 0; q0 < MAXC; q0 += G) {
        double pc[G], pE[G], pN[G], pW[G], pS[G], fq[G], nv[G];
        int kq[G], kd[G];
        Nb bq[G];
        bool act[G], ex[G];
#pragma unroll
        for (int u = 0; u < G; ++u) {
          const int q = q0 + u < MAXC ? q0 + u : MAXC - 1;
          int v = (q0 + u < MAXC) ? co[cc][q] : -1;
          // (more than 2 cells per thread and colour: the values derived here are
          // kept out of the loop, where they would hold registers)
          if constexpr (!PCREG) asm volatile("" : "+v"(v));
          kq[u] = hk + kof[cc][q];
          act[u] = v >= 0 && kq[u] > kbase && kq[u] <= kcap;
          kd[u] = v >> 15;
          bq[u] = nbrs_o(L, act[u] ? (v & 0x7fff) : W + 1);  // (an inactive slot loads a harmless cell)
          pc[u] = PCREG ? own[cc][q].pc : P[bq[u].o];
          pE[u] = P[bq[u].e];
          pN[u] = P[bq[u].n];
          pW[u] = P[bq[u].w];
          pS[u] = P[bq[u].s];
          fq[u] = FLDS ? F[bq[u].o] : fc[cc][FLDS ? 0 : q];
        }
#pragma unroll
        for (int u = 0; u < G; ++u) {
          const int q = q0 + u < MAXC ? q0 + u : MAXC - 1;
          ex[u] = false;
          CavMul m{};
          if (CASE == CAVITY) m = PRE ? cm[cc][PRE ? q : 0] : cav_mul(c, kd[u]);
          nv[u] = cell_compute<CASE>(c, own[cc][q], kd[u], pc[u], pE[u], pN[u], pW[u], pS[u], m, fq[u],
                                     !replay && kq[u] >= 2, tol, ex[u]);
        }
#pragma unroll
        for (int u = 0; u < G; ++u) {
          const int q = q0 + u < MAXC ? q0 + u : MAXC - 1;
          if (act[u] && q0 + u < MAXC) {
            cell_store<CASE>(P, flag, ck, ncell, bq[u], kd[u], nv[u], kq[u], kcap, ex[u], ml);
            own[cc][q] = {pW[u], pS[u], nv[u]};
          }
        }
      }
    }
    if (spt && col == colAB) {
      const int kB = kbase + ((H - (jc + ic + 1) + 2) >> 1) + 1, kA = kB + 1;
      if (kB > kbase && kB <= kcap) {
        const double b = cell_step<CASE>(c, P, flag, ck, ncell, bB, kindB, fB, ownB, kB, !replay && kB >= 2,
                                         kcap, ml, tol);
        if (kB < kcap) P[oC] = ((0.0 + b) + P[bA.o]) / 2;  // A at iteration kB
      }
      if (kA > kbase && kA <= kcap)
        cell_step<CASE>(c, P, flag, ck, ncell, bA, kindA, fA, ownA, kA, !replay && kA >= 2, kcap, ml, tol);
    }
    __syncthreads();
    // decisions (every thread the same)
    if (replay) {
      if (H >= Hend) break;
      continue;
    }
    if (pend > 0) {  // the lagged test (iterations in order)
      if (t == 0) flag[pend & (SMLEX_NF - 1)] = 0;  // (every thread read it before this barrier)
      if (fl == 0) K = pend;
      pend = 0;
    }
    if (K < 0 && H >= dmax && ((H - dmax) & 1) == 0) {  // iteration kc complete
      const int kc = ((H - dmax) >> 1) + 1;
      if (kc < max_iters) pend = kc;
    }
    if (K < 0 && H >= Hend) {  // every cell ran max_iters iterations: the last test now, then the cap
      if (pend > 0 && __builtin_amdgcn_readfirstlane(flag[pend & (SMLEX_NF - 1)]) == 0) K = pend;
      if (K < 0) {
        K = max_iters;
        break;
      }
    }
    if (K < 0) continue;
    pend = 0;
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
      refresh_all<CASE>(c, nx, ny, L, P);  // the field after iteration mstar's refresh
    }
    load_own();
    kbase = mstar;
    kcap = K;
    replay = true;
    Hend = dmax - 2 + 2 * (kcap - kbase - 1);
    H = -1;
  }

  // the final refresh (the reference's last applyPressureGhosts): ghosts from
  // the final interior with the solids as refreshed after iteration K-1, then
  // the solids
  refresh_all<CASE>(c, nx, ny, L, P);
  // the reported residual: max-norm of the final field (cavity-01.cpp:659-677)
  double m = 0.0;
#pragma unroll
  for (int cc = 0; cc < 2; ++cc)
#pragma unroll
    for (int q = 0; q < MAXC; ++q) {
      const int v = co[cc][q];
      if (v < 0) continue;
      const int o = v & 0x7fff, j = o / W, i = o - j * W;
      const Nb b = nbrs_o(L, o);
      m = fmax(m, residual_abs<CASE>(c, nx, ny, j, i, P[b.o], P[b.w], P[b.e], P[b.s], P[b.n],
                                     FLDS ? F[o] : fc[cc][FLDS ? 0 : q]));
    }
  if (spt) {
    m = fmax(m, residual_abs<CASE>(c, nx, ny, jc - 1, ic, P[bA.o], P[bA.w], P[bA.e], P[bA.s], P[bA.n], fA));
    m = fmax(m, residual_abs<CASE>(c, nx, ny, jc, ic + 1, P[bB.o], P[bB.w], P[bB.e], P[bB.s], P[bB.n], fB));
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
  // (more than 2 cells per thread and colour: p and the source in LDS)
  if ((long long)g.nx * g.ny > 4LL * SMLEX_THREADS && 2 * cells > SMLEX_CELLS) return false;
  const long long per_colour = ((long long)g.nx * g.ny + 1) / 2;
  if (cells > SMLEX_CELLS || per_colour > SMLEX_MAXC * SMLEX_THREADS || (g.nx + g.ny) / 2 + 8 >= SMLEX_NF)
    return false;
  if (cells > 0x7fff) return false;  // (a cell's LDS index: 15 bits)
  if (c.case_id == BACKSTEP) {  // a corner cell with fluid below and to the right
    if (!(c.step_i >= 2 && c.step_i <= g.nx - 1 && c.inlet_jmax >= 1 && c.inlet_jmax <= g.ny - 2)) return false;
  }
  return true;
}

size_t smlex_ck_doubles(int nx, int ny) { return (size_t)SMLEX_NCK * (nx + 2) * (ny + 2); }

int smlex_interval(int nx, int ny) {
  int m = 8;
  while (m < (nx + ny) / 6 + 2) m *= 2;  // (a power of two: iterations test it with a mask)
  return m;
}

void smlex_launch(int case_id, const Geo& g, const Coef& c, double* p, const double* f, const double* tolv,
                  int max_iters, double* ck, int* out_iters, double* out_res, hipStream_t st) {
  const long long per_colour = ((long long)g.nx * g.ny + 1) / 2;
  const int maxc = per_colour <= 2 * SMLEX_THREADS ? 2 : per_colour <= 4 * SMLEX_THREADS ? 4 : SMLEX_MAXC;
  int mlog = 0;
  while ((1 << mlog) < smlex_interval(g.nx, g.ny)) ++mlog;
#define CFD_SMLEX(CASE)                                                                                         \
  if (maxc == 2)                                                                                                \
    poisson_smlex_kernel<CASE, 2><<<1, SMLEX_THREADS, 0, st>>>(g, c, p, f, tolv, max_iters, ck, mlog, out_iters, out_res); \
  else if (maxc == 4)                                                                                           \
    poisson_smlex_kernel<CASE, 4><<<1, SMLEX_THREADS, 0, st>>>(g, c, p, f, tolv, max_iters, ck, mlog, out_iters, out_res); \
  else                                                                                                          \
    poisson_smlex_kernel<CASE, SMLEX_MAXC><<<1, SMLEX_THREADS, 0, st>>>(g, c, p, f, tolv, max_iters, ck, mlog, out_iters, out_res)
  if (case_id == CAVITY) { CFD_SMLEX(CAVITY); }
  else if (case_id == CHANNEL) { CFD_SMLEX(CHANNEL); }
  else { CFD_SMLEX(BACKSTEP); }
#undef CFD_SMLEX
}

}  // namespace cfd
