// small.hpp — the whole red-black SOR solve of a reference-sized grid in one
// persistent workgroup, the pressure field resident in LDS.
//
// The reference's own runs are tiny (cavity 63², channel 93×31, step 256×32,
// cavity-01.cpp:311-318, channel-01.cpp:289-290, backwards_step-01.cpp:323-324;
// BASELINE configs[0] is 128²): a multi-launch solve there is bound by launch
// and host-poll latency, not by the GPU. Here one workgroup of 16 waves holds
// p (rows 0..ny+1, columns 0..nx+1, (nx+2)(ny+2) doubles <= SMALL_CELLS, up to
// 158 KiB of LDS) and runs every iteration of the solve with barriers between
// the phases of the reference's iteration, testing the stop rule on the device:
//   red half-sweep (i+j even) | black half-sweep | [open cases: ghost rows /
//   columns, then solid cells, from the swept field] | max-norm residual.
// The same operations per cell in the same order as the multi-launch kernels
// and the oracle's red-black restatement (oracle/cfd_oracle.c sor_iteration,
// pressure_ghosts, residual_*), so the result is bit-identical to both.
//
// Work split: the cells of each colour are numbered row by row and dealt to
// the 1024 threads round-robin once, at launch (each thread keeps its cells'
// (j, i) and source values in registers), so every lane of every wave works in
// every half-sweep. The residual phase is skipped where the reference's loop
// cannot stop: on iterations it does not test (check_every), and for the
// cavity wherever the proof-mode test of kernels.hpp (proof_ratio) settles
// "some cell has |r| > tol" from the black updates, with each cell's own
// stencil values as P (a flag per iteration, no reduction).
#pragma once

#include "kernels.hpp"

namespace cfd {

constexpr int SMALL_CELLS = 20224;  // doubles of LDS for p: 158 KiB
constexpr int SMALL_THREADS = 1024;
constexpr int SMALL_WAVES = SMALL_THREADS / 64;
constexpr int SMALL_MAXC = 10;      // cells of one colour per thread: ceil((SMALL_CELLS / 2) / 1024)

// MAXC: cells of one colour per thread, >= ceil(cells of a colour / 1024)
// (2: up to 2048 per colour, e.g. 63^2, 93x31; 4: 256x32, 90^2; 10: any grid
// that fits the LDS)
template <int CASE, int MAXC>
__global__ __launch_bounds__(SMALL_THREADS) void poisson_small_kernel(Geo g, Coef c, double* __restrict__ p,
                                                                      const double* __restrict__ f,
                                                                      const double* __restrict__ tolv, int max_iters,
                                                                      int check_every, int* __restrict__ out_iters,
                                                                      double* __restrict__ out_res) {
  __shared__ double P[SMALL_CELLS];
  // per-iteration slots, rotating over three: iteration it uses slot it % 3 and
  // clears slot (it + 1) % 3 after its red half-sweep. That slot's last reads
  // were in iteration it - 2, and every wave has passed iteration it - 1's
  // barriers since, so no wave can still read it (two slots would race: a
  // lagging wave reading iteration it - 1's slot after thread 0 cleared it)
  __shared__ unsigned long long rmax_slot[3];  // max|r| of the iteration
  __shared__ int proven[3];                    // proof-mode: some cell proved |r| > tol
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int nx = g.nx, ny = g.ny, W = nx + 2;
  auto gidx = [&](int j, int i) { return (size_t)(j - g.row_lo) * (size_t)g.pitch + (size_t)i; };
  for (int j = w; j <= ny + 1; j += SMALL_WAVES)
    for (int i = lane; i <= nx + 1; i += 64) P[j * W + i] = p[gidx(j, i)];

  // this thread's cells of colour col (i + j even: red), in the order of
  // their numbering (row by row); non-fluid cells of the step are skipped
  // (the source values too while they fit the registers; larger grids read
  // them from global memory, cache-resident)
  constexpr bool FREG = MAXC <= 4;
  // cavity grids of up to 2 cells per thread and colour (the reference's 63^2):
  // each cell's omega / neighbour_count and its indicators as multipliers
  // (1.0 / 0.0: x * 0.0 == copysign(0, x), the reference's 0 * x, for finite
  // x), so the update is straight-line (sor_update<CAVITY>'s operations)
  constexpr bool PRE = CASE == CAVITY && MAXC <= 2;
  int cell[2][MAXC];  // (j << 16) | i, -1: none
  double fc[2][FREG ? MAXC : 1];
  double com[2][PRE ? MAXC : 1], cme[2][PRE ? MAXC : 1], cmw[2][PRE ? MAXC : 1], cmn[2][PRE ? MAXC : 1];
#pragma unroll
  for (int col = 0; col < 2; ++col) {
#pragma unroll
    for (int q = 0; q < MAXC; ++q) {
      const int e = t + q * SMALL_THREADS;  // (MAXC x 1024 >= cells of a colour)
      int v = -1;
      double fv = 0.0;
      {
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
        if (j <= ny && i <= nx && (CASE != BACKSTEP || is_fluid(c, nx, ny, j, i))) {
          v = (j << 16) | i;
          fv = f[gidx(j, i)];
        }
      }
      cell[col][q] = v;
      if constexpr (FREG) fc[col][q] = fv;
      if constexpr (PRE) {
        const int j = v >> 16, i = v & 0xffff;
        const int ee = i < nx, ew = i > 1, en = j < ny;
        double o1 = c.om_nc[1], o2 = c.om_nc[2], o3 = c.om_nc[3], o4 = c.om_nc[4];
        const int n = ee + ew + en + 1;
        com[col][q] = n == 4 ? o4 : n == 3 ? o3 : n == 2 ? o2 : o1;
        cme[col][q] = ee ? 1.0 : 0.0;
        cmw[col][q] = ew ? 1.0 : 0.0;
        cmn[col][q] = en ? 1.0 : 0.0;
      }
    }
  }
  if (t < 3) {
    rmax_slot[t] = 0ull;
    proven[t] = 0;
  }
  const double tol = tolv[0];
  // proof-mode test (cavity): per four-neighbour black cell, from its own
  // stencil: |p' - p| |K| (1 - 2^-38) > tol + 2^-43 (idx2 (P + h^2 |f|)(1 + 2^-40) + |f|)
  // with P = max of the six values it involves (kernels.hpp proof_ratio)
  const bool proof = CASE == CAVITY && c.proof_k > 0.0;
  const double kc = c.proof_k * (1.0 - 0x1p-38);
  double res = tolv[1];  // the loop's primed value (cavity-01.cpp:618, channel-01.cpp:649)
  int it = 0, sl = 0;  // sl = it % 3
  __syncthreads();
  // cavity-01.cpp:635 / channel-01.cpp:652 / backwards_step-01.cpp:893
  while (res > tol && it < max_iters) {
    ++it;
    sl = (sl == 2) ? 0 : sl + 1;
    const int sl_next = (sl == 2) ? 0 : sl + 1;
    // tested on check_every multiples and at the cap, like the multi-launch
    // solve; the cap always evaluates the residual (it is reported)
    const bool tested = it % check_every == 0 || it == max_iters;
    const bool try_proof = proof && tested && it < max_iters;
    bool pf = false;
#pragma unroll
    for (int col = 0; col < 2; ++col) {  // red: i+j even, then black
#pragma unroll
      for (int q = 0; q < MAXC; ++q) {
        const int v = cell[col][q];
        if (v >= 0) {
          const int j = v >> 16, i = v & 0xffff;
          const int o = j * W + i;
          const double old = P[o], pw = P[o - 1], pe = P[o + 1], ps = P[o - W], pn = P[o + W];
          const double fq = FREG ? fc[col][FREG ? q : 0] : f[gidx(j, i)];
          double nv;
          if constexpr (PRE) {
            const int qq = PRE ? q : 0;
            nv = old * c.one_m_omega +
                 com[col][qq] * ((pe * cme[col][qq] + pw * cmw[col][qq]) + (pn * cmn[col][qq] + ps) - fq * c.h2);
          } else {
            nv = sor_update<CASE>(c, nx, ny, j, i, old, pw, pe, ps, pn, fq);
          }
          P[o] = nv;
          if (col == 1 && try_proof && i > 1 && i < nx && j < ny) {
            const double pc = fmax(fmax(fmax(fabs(old), fabs(nv)), fmax(fabs(pw), fabs(pe))), fmax(fabs(ps), fabs(pn)));
            const double af = fabs(fq);
            const double rhs = tol + 0x1p-43 * (c.idx2 * ((pc + c.h2 * af) * (1.0 + 0x1p-40)) + af);
            pf = pf || fabs(nv - old) * kc > rhs;
          }
        }
      }
      if (col == 0) {
        if (t == 0) {  // the next iteration's slots (last read in iteration it - 2)
          rmax_slot[sl_next] = 0ull;
          proven[sl_next] = 0;
        }
      } else if (pf) {
        proven[sl] = 1;  // (any proving lane: the same value)
      }
      __syncthreads();
    }
    if (CASE != CAVITY) {
      // channel-01.cpp:531-541 / backwards_step-01.cpp:685-706: ghost columns
      // and rows from the swept interior (corners untouched)
      for (int e = t; e < ny + nx; e += SMALL_THREADS) {
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
      if (CASE == BACKSTEP) {  // backwards_step-01.cpp:708-738: solids next to fluid
        for (int j = 1 + w; j <= ny; j += SMALL_WAVES)
          for (int i = 1 + lane; i <= nx; i += 64) {
            if (is_fluid(c, nx, ny, j, i)) continue;
            const int o = j * W + i;
            double out;
            if (refresh_value<CASE>(c, nx, ny, j, i, P[o], P[o - 1], P[o + 1], P[o - W], P[o + W], out)) P[o] = out;
          }
        __syncthreads();
      }
    }
    const bool exact = tested && !(try_proof && proven[sl] != 0);  // block-uniform
    if (exact) {
      // max-norm residual of the iteration (cavity-01.cpp:659-677,
      // channel-01.cpp:672-681, backwards_step-01.cpp:916-930): one LDS
      // atomic per wave into this iteration's slot
      double m = 0.0;
#pragma unroll
      for (int col = 0; col < 2; ++col)
#pragma unroll
        for (int q = 0; q < MAXC; ++q) {
          const int v = cell[col][q];
          if (v >= 0) {
            const int j = v >> 16, i = v & 0xffff;
            const int o = j * W + i;
            const double fq = FREG ? fc[col][FREG ? q : 0] : f[gidx(j, i)];
            m = fmax(m, residual_abs<CASE>(c, nx, ny, j, i, P[o], P[o - 1], P[o + 1], P[o - W], P[o + W], fq));
          }
        }
      m = wave_max(m);
      if (lane == 0) atomicMax(&rmax_slot[sl], (unsigned long long)__double_as_longlong(m));
      __syncthreads();
      const double rk = __longlong_as_double((long long)rmax_slot[sl]);
      res = rk;
      if (t == 0 && !(res > tol && it < max_iters)) {
        *out_iters = it;
        *out_res = rk;
      }
    } else {
      res = __builtin_huge_val();
    }
  }
  if (it == 0 && t == 0) {
    *out_iters = 0;
    *out_res = res;
  }
  __syncthreads();
  for (int j = w; j <= ny + 1; j += SMALL_WAVES)
    for (int i = lane; i <= nx + 1; i += 64) p[gidx(j, i)] = P[j * W + i];
}

}  // namespace cfd
