// bw_probe.hip — practical HBM ceiling for the SOR kernel's byte mix on this
// GPU: out[i] = a[i] + b[i] over fp64 arrays of the bench size (2 reads +
// 1 write per cell, like p_in + f -> p_out), with 16-B lanes, grid-stride.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256) void add2(const double2* __restrict__ a, const double2* __restrict__ b,
                                            double2* __restrict__ c, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const double2 x = a[i], y = b[i];
    c[i] = make_double2(x.x + y.x, x.y + y.y);
  }
}
__global__ __launch_bounds__(256) void read2(const double2* __restrict__ a, const double2* __restrict__ b,
                                             double* __restrict__ out, size_t n) {
  double s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const double2 x = a[i], y = b[i];
    s += x.x + y.y;
  }
  if (s == 12345.678) out[0] = s;
}

int main(int argc, char** argv) {
  const size_t cells = (size_t)4098 * 4112;
  const size_t n = cells / 2;
  double2 *a, *b, *c;
  hipMalloc(&a, n * 16); hipMalloc(&b, n * 16); hipMalloc(&c, n * 16);
  hipMemset(a, 0, n * 16); hipMemset(b, 0, n * 16); hipMemset(c, 0, n * 16);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  int grids[] = {1024, 2048, 4096, 8192, 16384, 65536};
  for (int gsz : grids) {
    for (int rep = 0; rep < 2; ++rep) add2<<<gsz, 256>>>(a, b, c, n);
    hipEventRecord(e0);
    const int R = 50;
    for (int rep = 0; rep < R; ++rep) add2<<<gsz, 256>>>(a, b, c, n);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / R;
    printf("add2  grid=%6d  %8.2f us  %7.1f GB/s (24 B/cell)\n", gsz, us, 24.0 * cells / (us * 1e-6) / 1e9);
    hipEventRecord(e0);
    for (int rep = 0; rep < R; ++rep) read2<<<gsz, 256>>>(a, b, (double*)c, n);
    hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("read2 grid=%6d  %8.2f us  %7.1f GB/s (16 B/cell)\n", gsz, ms * 1e3 / R, 16.0 * cells / (ms * 1e-3 / R) / 1e9);
  }
  return 0;
}
