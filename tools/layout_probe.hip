// layout_probe.hip — does a panel layout make the SOR march's traffic cheaper?
// Each wave marches a band of TH rows over a 120-column tile (2 fp64 per lane,
// 16-B loads of two arrays + one 16-B store per row), as poisson_wave_kernel
// does, with the rows either row-major (stride = pitch) or in 120-column
// panels stored contiguously (stride = 120). Traffic only, no arithmetic.
#include <hip/hip_runtime.h>
#include <cstdio>

template <bool PANEL>
__global__ __launch_bounds__(256) void march(const double* __restrict__ a, const double* __restrict__ b,
                                             double* __restrict__ c, int rows, int pitch, int ctiles, int nbands,
                                             int TH) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int tile = blockIdx.x * 4 + wv;
  if (tile >= ctiles * nbands) return;
  const int band = tile % nbands, ct = tile / nbands;
  if (lane >= 60) return;
  const int y0 = band * TH, y1 = min(y0 + TH, rows);
  size_t base, stride;
  if (PANEL) { base = (size_t)ct * rows * 120 + lane * 2; stride = 120; }
  else { base = (size_t)ct * 120 + lane * 2; stride = pitch; }
  double2 acc = make_double2(0, 0);
  for (int r = y0; r < y1; ++r) {
    const size_t o = base + (size_t)r * stride;
    const double2 x = *reinterpret_cast<const double2*>(a + o);
    const double2 y = *reinterpret_cast<const double2*>(b + o);
    *reinterpret_cast<double2*>(c + o) = make_double2(x.x + y.x, x.y + y.y);
  }
}

int main() {
  const int rows = 4098, pitch = 4112, ctiles = 35;
  const size_t n = (size_t)ctiles * 120 * rows + 64;
  double *a, *b, *c;
  (void)hipMalloc(&a, n * 8); (void)hipMalloc(&b, n * 8); (void)hipMalloc(&c, n * 8);
  (void)hipMemset(a, 0, n * 8); (void)hipMemset(b, 0, n * 8);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  for (int nb : {29, 58, 117, 234}) {
    const int TH = (rows + nb - 1) / nb;
    const int blocks = (ctiles * nb + 3) / 4;
    for (int pass = 0; pass < 2; ++pass) {
      for (int w = 0; w < 3; ++w) {
        if (pass) march<true><<<blocks, 256>>>(a, b, c, rows, pitch, ctiles, nb, TH);
        else march<false><<<blocks, 256>>>(a, b, c, rows, pitch, ctiles, nb, TH);
      }
      (void)hipEventRecord(e0);
      for (int w = 0; w < 50; ++w) {
        if (pass) march<true><<<blocks, 256>>>(a, b, c, rows, pitch, ctiles, nb, TH);
        else march<false><<<blocks, 256>>>(a, b, c, rows, pitch, ctiles, nb, TH);
      }
      (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1e3 / 50;
      printf("%s bands=%3d TH=%4d  %7.2f us  %6.1f GB/s\n", pass ? "panel   " : "rowmajor", nb, TH, us,
             24.0 * 4098 * 4098 / (us * 1e-6) / 1e9);
    }
  }
  return 0;
}
