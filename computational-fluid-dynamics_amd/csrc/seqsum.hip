// seqsum.hip — sequential sums in the reference's loop order, bit for bit.
//
// The reference-order mode (ordering = CFD_ORDER_LEX) reproduces the
// reference's own sums: the channel's / step's source mean (channel-01.cpp:
// 620-628, backwards_step-01.cpp:843-866) once per timestep and the kinetic
// energy of the statistics (cavity-01.cpp:750-755). Each partial sum is
// rounded before the next term is added, so the sum is one chain of dependent
// fp64 adds: its time is the add latency times the terms, whatever the
// parallelism around it. The kernel therefore keeps the chain fed and nothing
// else on it: one 512-thread workgroup, waves 1-7 stage the terms of the next
// chunk (SEQ_CHUNK terms in loop order, a solid cell as -0.0, which leaves
// every sum unchanged: x + -0.0 == x, -0.0 + -0.0 == -0.0, as skipping it
// does) into LDS while wave 0 adds the current chunk, reading the terms as
// broadcast LDS loads (every lane the same address) one batch ahead of the
// adds. One barrier per chunk.
#include "seqsum.hpp"

namespace cfd {

namespace {

constexpr int SEQ_THREADS = 512;
constexpr int SEQ_CHUNK = 4096;  // terms per LDS chunk; two chunks (64 KiB)
constexpr int SEQ_BATCH = 32;    // terms the adder has in registers, the next batch in flight

__global__ __launch_bounds__(SEQ_THREADS) void seq_sum_kernel(Geo g, Coef c, const double* __restrict__ a,
                                                              const double* __restrict__ b, int mode,
                                                              double* __restrict__ out, int accumulate) {
  __shared__ double buf[2][SEQ_CHUNK];
  const int t = threadIdx.x, w = t >> 6;
  const int ja = max(g.j0, 1), jb = min(g.j1, g.ny);
  const int nx = g.nx;
  const long long n = (long long)max(0, jb - ja + 1) * nx;  // terms: q -> (ja + q / nx, 1 + q % nx)
  const int nch = (int)((n + SEQ_CHUNK - 1) / SEQ_CHUNK);
  // waves 1..7: the terms of chunk ch into dst, in loop order
  auto produce = [&](int ch, double* dst) {
    const long long q0 = (long long)ch * SEQ_CHUNK;
    int e = t - 64;
    long long q = q0 + e;
    int jq = (int)(q / nx);
    int i = 1 + (int)(q - (long long)jq * nx);
    constexpr int STEP = SEQ_THREADS - 64;  // (448 < nx is not assumed: the row advance loops)
    for (; e < SEQ_CHUNK; e += STEP) {
      double tv = -0.0;
      if (q < n) {
        const int j = ja + jq;
        const size_t o = at(g, j, i);
        const double v = (mode == 0) ? a[o] : 0.5 * (a[o] * a[o] + b[o] * b[o]);
        tv = is_fluid(c, nx, g.ny, j, i) ? v : -0.0;
      }
      dst[e] = tv;
      q += STEP;
      i += STEP;
      while (i > nx) {
        i -= nx;
        ++jq;
      }
    }
  };
  if (w > 0 && nch > 0) produce(0, buf[0]);
  double s = accumulate ? out[0] : 0.0;
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    if (w > 0) {
      if (ch + 1 < nch) produce(ch + 1, buf[(ch + 1) & 1]);
    } else {
      // the chain: every lane adds the same terms (broadcast reads), in order;
      // the chunk's tail past n holds -0.0 (no change), so whole batches run
      const double* src = buf[ch & 1];
      const long long left = n - (long long)ch * SEQ_CHUNK;
      const int len = (int)(left < SEQ_CHUNK ? (left + SEQ_BATCH - 1) / SEQ_BATCH * SEQ_BATCH : SEQ_CHUNK);
      double d[SEQ_BATCH], e[SEQ_BATCH];
#pragma unroll
      for (int u = 0; u < SEQ_BATCH; ++u) d[u] = src[u];
      for (int k = 0; k < len; k += SEQ_BATCH) {
        const int kn = (k + SEQ_BATCH < len) ? k + SEQ_BATCH : k;  // (the last batch reloads itself: unused)
#pragma unroll
        for (int u = 0; u < SEQ_BATCH; ++u) e[u] = src[kn + u];
#pragma unroll
        for (int u = 0; u < SEQ_BATCH; ++u) s += d[u];
#pragma unroll
        for (int u = 0; u < SEQ_BATCH; ++u) d[u] = e[u];
      }
    }
    __syncthreads();
  }
  if (t == 0) out[0] = s;
}

}  // namespace

void seq_sum_launch(const Geo& g, const Coef& c, const double* a, const double* b, int mode, double* out,
                    int accumulate, hipStream_t st) {
  seq_sum_kernel<<<1, SEQ_THREADS, 0, st>>>(g, c, a, b, mode, out, accumulate);
}

}  // namespace cfd
