// add_chain.hip — latency floor of a dependent fp64 add chain on gfx950 (the
// reference order's sequential sums, seqsum.hip). One workgroup; wave 0 adds
// N terms into one running sum, each add waiting for the previous one:
//   reg    : terms already in VGPRs (the pure v_add_f64 dependency chain)
//   lane0  : the same with only lane 0 active (does a partial EXEC shorten it?)
//   sgpr   : terms in SGPRs (readfirstlane'd), v_add_f64 v, s, v
//   lds    : terms broadcast-read from LDS one batch ahead of the adds
//   readlane: one coalesced LDS read per 64 terms, v_readlane into SGPRs
// Prints ns and cycles per add (hipEvent wall time of the launch / N).
// build: hipcc -O3 --offload-arch=gfx950 tools/add_chain.hip -o tools/add_chain
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                              \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

constexpr int B = 32;

template <int MODE>
__global__ __launch_bounds__(256) void chain(const double* __restrict__ a, int reps, double* out,
                                             long long* cyc) {
  __shared__ double buf[4096];
  const int t = threadIdx.x;
  for (int k = t; k < 4096; k += 256) buf[k] = a[k];
  __syncthreads();
  if (t >= 64) return;
  double s = 0.0;
  const long long t0 = clock64();
  if constexpr (MODE == 0 || MODE == 1) {
    double r[B];
#pragma unroll
    for (int u = 0; u < B; ++u) r[u] = buf[u + t];
    if (MODE == 1 && t != 0) return;
    for (int q = 0; q < reps; ++q) {
#pragma unroll
      for (int u = 0; u < B; ++u) s += r[u];
      asm volatile("" : "+v"(s));
    }
  } else if constexpr (MODE == 2) {
    double r[B];
#pragma unroll
    for (int u = 0; u < B; ++u) {
      const double v = buf[u];
      r[u] = __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)),
                              __builtin_amdgcn_readfirstlane(__double2loint(v)));
    }
    for (int q = 0; q < reps; ++q) {
#pragma unroll
      for (int u = 0; u < B; ++u) s += r[u];
      asm volatile("" : "+v"(s));
    }
  } else if constexpr (MODE == 4) {  // one coalesced LDS read per 64 terms, terms taken by v_readlane
    double v = buf[t], vn;
    for (int q = 0; q < reps / 2; ++q) {
      vn = buf[(((q + 1) * 64) & 4095) + t];
      asm volatile("" : "+v"(s)::"memory");
#pragma unroll
      for (int u = 0; u < 64; ++u)
        s += __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), u),
                              __builtin_amdgcn_readlane(__double2loint(v), u));
      v = vn;
    }
  } else {  // LDS broadcast reads, next batch in flight during the adds
    double d[B], e[B];
#pragma unroll
    for (int u = 0; u < B; ++u) d[u] = buf[u];
    for (int q = 0; q < reps; ++q) {
      const int base = ((q + 1) * B) & 4095;
#pragma unroll
      for (int u = 0; u < B; ++u) e[u] = buf[base + u];
      asm volatile("" ::: "memory");
#pragma unroll
      for (int u = 0; u < B; ++u) s += d[u];
      asm volatile("" : "+v"(s));
#pragma unroll
      for (int u = 0; u < B; ++u) d[u] = e[u];
    }
  }
  const long long t1 = clock64();
  if (t == 0) {
    out[0] = s;
    cyc[0] = t1 - t0;
  }
}

int main() {
  const int reps = 20000;
  const long long n = (long long)reps * B;
  std::vector<double> h(4096);
  for (int k = 0; k < 4096; ++k) h[k] = 1e-3 * ((k * 2654435761u) % 1000003) - 500.0;
  double *a, *out;
  long long* cyc;
  CK(hipMalloc(&a, 4096 * sizeof(double)));
  CK(hipMalloc(&out, 8));
  CK(hipMalloc(&cyc, 8));
  CK(hipMemcpy(a, h.data(), 4096 * sizeof(double), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[5] = {"reg", "lane0", "sgpr", "lds", "readlane"};
  std::printf("{\"adds\": %lld, \"modes\": {", n);
  for (int m = 0; m < 5; ++m) {
    for (int rep = 0; rep < 2; ++rep) {  // (second run timed)
      CK(hipEventRecord(e0));
      if (m == 0) chain<0><<<1, 256>>>(a, reps, out, cyc);
      if (m == 1) chain<1><<<1, 256>>>(a, reps, out, cyc);
      if (m == 2) chain<2><<<1, 256>>>(a, reps, out, cyc);
      if (m == 3) chain<3><<<1, 256>>>(a, reps, out, cyc);
      if (m == 4) chain<4><<<1, 256>>>(a, reps, out, cyc);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
    }
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    long long c = 0;
    CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
    std::printf("%s\"%s\": {\"ns_per_add\": %.3f, \"clock64_per_add\": %.2f}", m ? ", " : "", names[m],
                ms * 1e6 / n, (double)c / n);
  }
  std::printf("}}\n");
  return 0;
}
