// Practical HBM ceiling for the red-black launch's traffic shape: read two
// 4096^2 fp64 fields (p_in, f) and write one (p_out), 403 MB per launch - the
// algorithmic bytes bench.py prices the headline launch at. Variants: plain
// grid-stride double2 triad, and a row-march with the SOR launch's geometry
// (one wave per 128-column x th-row band, 16-B lanes, 4 rows prefetched,
// nontemporal stores). Median of 200 launches each.
// Build: hipcc --offload-arch=gfx950 -O3 tools/hbm_ceiling.hip -o tools/hbm_ceiling
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));

// NT: streamed (nontemporal) stores, as the SOR kernels' store_row_pair
template <bool NT>
__global__ __launch_bounds__(256) void triad(const double2* __restrict__ a, const double2* __restrict__ b,
                                             double2* __restrict__ c, size_t n2) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) {
    const double2 x = a[i], y = b[i];
    if (NT) {
      d2v v = {x.x + 0.5 * y.x, x.y + 0.5 * y.y};
      __builtin_nontemporal_store(v, reinterpret_cast<d2v*>(c + i));
    } else {
      c[i] = make_double2(x.x + 0.5 * y.x, x.y + 0.5 * y.y);
    }
  }
}

// each wave: 128 columns (2 per lane) x th rows, marching down with PD rows in flight
template <int PD>
__global__ __launch_bounds__(256, 2) void march(const double* __restrict__ a, const double* __restrict__ b,
                                                double* __restrict__ c, int nx, int ny, int th, int nbands) {
  const int lane = threadIdx.x & 63;
  const int wv = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int ct = wv / nbands, band = wv % nbands;
  const int col = ct * 128 + 2 * lane;
  const int y0 = band * th, y1 = min(y0 + th, ny);
  if (col >= nx || y0 >= y1) return;
  double2 ra[PD], rb[PD];
#pragma unroll
  for (int q = 0; q < PD; ++q) {
    const int y = min(y0 + q, y1 - 1);
    ra[q] = *reinterpret_cast<const double2*>(a + (size_t)y * nx + col);
    rb[q] = *reinterpret_cast<const double2*>(b + (size_t)y * nx + col);
  }
  for (int y = y0; y < y1; y += PD) {
#pragma unroll
    for (int q = 0; q < PD; ++q) {
      const double2 x = ra[q], z = rb[q];
      const int yn = min(y + q + PD, y1 - 1);
      ra[q] = *reinterpret_cast<const double2*>(a + (size_t)yn * nx + col);
      rb[q] = *reinterpret_cast<const double2*>(b + (size_t)yn * nx + col);
      d2v v = {x.x + 0.5 * z.x, x.y + 0.5 * z.y};
      if (y + q < y1) __builtin_nontemporal_store(v, reinterpret_cast<d2v*>(c + (size_t)(y + q) * nx + col));
    }
  }
}

// the same march with SOR-like arithmetic per row: 8 row updates of ~10 fp64
// VALU each (4 sweeps x red/black) over a carried 8-row x 2-column window,
// PD rows of both inputs in flight (what the 4-sweep launch does per march step,
// without its fill rows and halo lanes)
template <int PD>
__global__ __launch_bounds__(256, 2) void march_compute(const double* __restrict__ a, const double* __restrict__ b,
                                                        double* __restrict__ c, int nx, int ny, int th, int nbands,
                                                        double om, double h2) {
  const int lane = threadIdx.x & 63;
  const int wv = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int ct = wv / nbands, band = wv % nbands;
  const int col = ct * 128 + 2 * lane;
  const int y0 = band * th, y1 = min(y0 + th, ny);
  if (col >= nx || y0 >= y1) return;
  double2 ra[PD], rb[PD], w[9], fr[8];
#pragma unroll
  for (int q = 0; q < 9; ++q) w[q] = make_double2(0.0, 0.0);
#pragma unroll
  for (int q = 0; q < 8; ++q) fr[q] = make_double2(0.0, 0.0);
#pragma unroll
  for (int q = 0; q < PD; ++q) {
    const int y = min(y0 + q, y1 - 1);
    ra[q] = *reinterpret_cast<const double2*>(a + (size_t)y * nx + col);
    rb[q] = *reinterpret_cast<const double2*>(b + (size_t)y * nx + col);
  }
  for (int y = y0; y < y1; y += PD) {
#pragma unroll
    for (int q = 0; q < PD; ++q) {
      // shift the window (compile-time: the unrolled loop renames registers)
#pragma unroll
      for (int k = 8; k > 0; --k) w[k] = w[k - 1];
#pragma unroll
      for (int k = 7; k > 0; --k) fr[k] = fr[k - 1];
      w[0] = ra[q];
      fr[0] = rb[q];
      const int yn = min(y + q + PD, y1 - 1);
      ra[q] = *reinterpret_cast<const double2*>(a + (size_t)yn * nx + col);
      rb[q] = *reinterpret_cast<const double2*>(b + (size_t)yn * nx + col);
#pragma unroll
      for (int k = 1; k <= 8; ++k) {
        const double l = __shfl_up(w[k].y, 1);  // (the DPP neighbour of the SOR kernels)
        w[k].x = (1.0 - om) * w[k].x + om * 0.25 * ((l + w[k].y) + (w[k - 1].x + w[k + 1 < 9 ? k + 1 : 8].x) - h2 * fr[k - 1].x);
      }
      d2v v = {w[8].x, w[8].y};
      if (y + q < y1) __builtin_nontemporal_store(v, reinterpret_cast<d2v*>(c + (size_t)(y + q) * nx + col));
    }
  }
}

template <class F>
static float time_it(F launch, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 5; ++i) launch();
  std::vector<float> t;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main() {
  const int nx = 4096, ny = 4096;
  const size_t n = (size_t)nx * ny, bytes = 3 * n * sizeof(double);
  double *a, *b, *c;
  CK(hipMalloc(&a, n * 8));
  CK(hipMalloc(&b, n * 8));
  CK(hipMalloc(&c, n * 8));
  CK(hipMemset(a, 0, n * 8));
  CK(hipMemset(b, 0, n * 8));
  printf("{\"bytes_per_launch\": %zu, \"results\": [\n", bytes);
  bool first = true;
  auto report = [&](const char* name, float ms) {
    printf("%s{\"variant\": \"%s\", \"us\": %.2f, \"GBs\": %.1f, \"frac_of_8000\": %.4f}\n", first ? "" : ",", name,
           ms * 1e3, bytes / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / 1e9 / 8000.0);
    first = false;
  };
  for (int blocks : {1024, 2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, sizeof nm, "triad grid-stride %d blocks", blocks);
    report(nm, time_it([&] { triad<false><<<blocks, 256>>>((const double2*)a, (const double2*)b, (double2*)c, n / 2); }, 200));
    snprintf(nm, sizeof nm, "triad grid-stride %d blocks, nt stores", blocks);
    report(nm, time_it([&] { triad<true><<<blocks, 256>>>((const double2*)a, (const double2*)b, (double2*)c, n / 2); }, 200));
  }
  for (int th : {32, 64, 128}) {
    const int nbands = (ny + th - 1) / th, waves = 32 * nbands;
    char nm[64];
    snprintf(nm, sizeof nm, "march th=%d (%d waves), nt stores", th, waves);
    report(nm, time_it([&] { march<4><<<(waves + 3) / 4, 256>>>(a, b, c, nx, ny, th, nbands); }, 200));
  }
  for (int th : {64, 128}) {
    const int nbands = (ny + th - 1) / th, waves = 32 * nbands;
    char nm[96];
    snprintf(nm, sizeof nm, "march+8 updates th=%d (%d waves), PD 4", th, waves);
    report(nm, time_it([&] { march_compute<4><<<(waves + 3) / 4, 256>>>(a, b, c, nx, ny, th, nbands, 1.7, 1e-6); }, 200));
    snprintf(nm, sizeof nm, "march+8 updates th=%d (%d waves), PD 8", th, waves);
    report(nm, time_it([&] { march_compute<8><<<(waves + 3) / 4, 256>>>(a, b, c, nx, ny, th, nbands, 1.7, 1e-6); }, 200));
  }
  printf("]}\n");
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(c));
  return 0;
}
