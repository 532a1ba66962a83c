// small.hpp — the whole red-black SOR solve of a reference-sized grid in one
// persistent workgroup, the pressure field resident in LDS.
//
// The reference's own runs are tiny (cavity 63², channel 93×31, step 256×32,
// cavity-01.cpp:311-318, channel-01.cpp:289-290, backwards_step-01.cpp:323-324;
// BASELINE configs[0] is 128²): a multi-launch solve there is bound by launch
// and host-poll latency, not by the GPU. Here one workgroup of 16 waves holds
// p (rows 0..ny+1, columns 0..nx+1, (nx+2)(ny+2) doubles <= SMALL_CELLS, up to
// 160 KiB of LDS) and runs every iteration of the solve with barriers between
// the phases of the reference's iteration, testing the stop rule on the device:
//   red half-sweep (i+j even) | black half-sweep | [open cases: ghost rows /
//   columns, then solid cells, from the swept field] | max-norm residual.
// The same operations per cell in the same order as the multi-launch kernels
// and the oracle's red-black restatement (oracle/cfd_oracle.c sor_iteration,
// pressure_ghosts, residual_*), so the result is bit-identical to both; the
// source f is read from global memory (read-only, cache resident).
#pragma once

#include "kernels.hpp"

namespace cfd {

constexpr int SMALL_CELLS = 20224;  // doubles of LDS for p (and f when both fit): 158 KiB
constexpr int SMALL_THREADS = 1024;
constexpr int SMALL_WAVES = SMALL_THREADS / 64;

// Cells are walked without divisions: wave w takes rows w+1, w+1+16, ...; a
// lane takes columns 2*lane (one colour) or lane (both) + multiples of 128 / 64.
// FL: the source f in LDS next to p (grids of up to SMALL_CELLS / 2 cells), or
// read from global memory.
template <int CASE, bool FL>
__global__ __launch_bounds__(SMALL_THREADS) void poisson_small_kernel(Geo g, Coef c, double* __restrict__ p,
                                                                      const double* __restrict__ f,
                                                                      const double* __restrict__ tolv, int max_iters,
                                                                      int check_every, int* __restrict__ out_iters,
                                                                      double* __restrict__ out_res) {
  __shared__ double P[SMALL_CELLS];
  __shared__ unsigned long long rmax[2];  // |r| >= 0: its bits order like the values
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int nx = g.nx, ny = g.ny, W = nx + 2;
  const int ncell = (ny + 2) * W;
  double* F = P + ncell;  // FL only
  auto gidx = [&](int j, int i) { return (size_t)(j - g.row_lo) * (size_t)g.pitch + (size_t)i; };
  for (int j = w; j <= ny + 1; j += SMALL_WAVES)
    for (int i = lane; i <= nx + 1; i += 64) {
      P[j * W + i] = p[gidx(j, i)];
      if (FL) F[j * W + i] = f[gidx(j, i)];
    }
  auto fv = [&](int j, int i) { return FL ? F[j * W + i] : f[gidx(j, i)]; };
  if (t < 2) rmax[t] = 0ull;
  const double tol = tolv[0];
  double res = tolv[1];  // the loop's primed value (cavity-01.cpp:618, channel-01.cpp:649)
  int it = 0;
  __syncthreads();
  // cavity-01.cpp:635 / channel-01.cpp:652 / backwards_step-01.cpp:893
  while (res > tol && it < max_iters) {
    ++it;
    for (int color = 0; color < 2; ++color) {  // red: i+j even, then black
      for (int j = 1 + w; j <= ny; j += SMALL_WAVES)
        for (int i = 1 + ((j + 1 + color) & 1) + 2 * lane; i <= nx; i += 128) {
          if (CASE == BACKSTEP && !is_fluid(c, nx, ny, j, i)) continue;
          const int o = j * W + i;
          P[o] = sor_update<CASE>(c, nx, ny, j, i, P[o], P[o - 1], P[o + 1], P[o - W], P[o + W], fv(j, i));
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
    // max-norm residual of the iteration (cavity-01.cpp:659-677,
    // channel-01.cpp:672-681, backwards_step-01.cpp:916-930): one LDS atomic
    // per wave into this iteration's slot; the other slot is cleared for the next
    double m = 0.0;
    for (int j = 1 + w; j <= ny; j += SMALL_WAVES)
      for (int i = 1 + lane; i <= nx; i += 64) {
        if (CASE == BACKSTEP && !is_fluid(c, nx, ny, j, i)) continue;
        const int o = j * W + i;
        m = fmax(m, residual_abs<CASE>(c, nx, ny, j, i, P[o], P[o - 1], P[o + 1], P[o - W], P[o + W], fv(j, i)));
      }
    m = wave_max(m);
    if (lane == 0) atomicMax(&rmax[it & 1], (unsigned long long)__double_as_longlong(m));
    if (t == 0) rmax[(it + 1) & 1] = 0ull;
    __syncthreads();
    // tested on check_every multiples and at the cap, like the multi-launch solve
    const double rk = __longlong_as_double((long long)rmax[it & 1]);
    res = (it % check_every == 0 || it == max_iters) ? rk : __builtin_huge_val();
    if (t == 0 && !(res > tol && it < max_iters)) {
      *out_iters = it;
      *out_res = rk;
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
