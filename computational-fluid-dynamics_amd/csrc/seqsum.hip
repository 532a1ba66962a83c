// seqsum.hip — sequential sums in the reference's loop order, bit for bit.
//
// The reference-order mode (ordering = CFD_ORDER_LEX) reproduces the
// reference's own sums: the channel's / step's source mean (channel-01.cpp:
// 620-628, backwards_step-01.cpp:843-866) once per timestep and the kinetic
// energy of the statistics (cavity-01.cpp:750-755). Each partial sum is
// rounded before the next term is added, so the sum is one chain of dependent
// fp64 adds: its time is the add latency times the terms, whatever the
// parallelism around it. The kernel therefore keeps the chain fed and nothing
// else on it: one 256-thread workgroup (one wave per SIMD), waves 1-3 stage
// the terms of the next chunk (SEQ_CHUNK terms in loop order, a solid cell as
// -0.0, which leaves every sum unchanged: x + -0.0 == x, -0.0 + -0.0 == -0.0,
// as skipping it does) into LDS, SEQ_LOADS global loads in flight per thread,
// while wave 0, alone on its SIMD, adds the current chunk: broadcast LDS loads
// (every lane the same address) of the next batch are issued before the adds
// of this one (a compiler barrier keeps them there; otherwise the loads sink
// to their use and every batch waits for its own LDS round trip), in fully
// unrolled blocks (no register copies). One barrier per chunk. The dependent
// v_add_f64 chain itself takes 2.9 ns per add on MI355X (tools/add_chain.hip,
// profiles/r5/add_chain.json).
#include "seqsum.hpp"

namespace cfd {

namespace {

constexpr int SEQ_THREADS = 256;  // wave 0 adds; waves 1-3 stage (one wave per SIMD)
constexpr int SEQ_CHUNK = 8192;   // terms per LDS chunk; two chunks (128 KiB)
constexpr int SEQ_BATCH = 32;     // terms the adder has in registers, the next batch in flight
constexpr int SEQ_BLOCK = 1024;   // terms per unrolled block of the adder (a multiple of SEQ_BATCH)
static_assert(SEQ_CHUNK % SEQ_BLOCK == 0 && SEQ_BLOCK % SEQ_BATCH == 0, "seqsum blocking");
constexpr int SEQ_LOADS = 8;      // global loads in flight per staging thread

__global__ __launch_bounds__(SEQ_THREADS) void seq_sum_kernel(Geo g, Coef c, const double* __restrict__ a,
                                                              const double* __restrict__ b, int mode,
                                                              double* __restrict__ out, int accumulate) {
  __shared__ double buf[2][SEQ_CHUNK];
  const int t = threadIdx.x, w = t >> 6;
  const int ja = max(g.j0, 1), jb = min(g.j1, g.ny);
  const int nx = g.nx;
  const long long n = (long long)max(0, jb - ja + 1) * nx;  // terms: q -> (ja + q / nx, 1 + q % nx)
  const int nch = (int)((n + SEQ_CHUNK - 1) / SEQ_CHUNK);
  // waves 1..3: the terms of chunk ch into dst, in loop order; each thread
  // issues SEQ_LOADS loads before it writes any of them
  auto produce = [&](int ch, double* dst) {
    constexpr int STEP = SEQ_THREADS - 64;
    const long long q0 = (long long)ch * SEQ_CHUNK;
    for (int e0 = t - 64; e0 < SEQ_CHUNK; e0 += STEP * SEQ_LOADS) {
      double v[SEQ_LOADS];
      bool ok[SEQ_LOADS];
#pragma unroll
      for (int u = 0; u < SEQ_LOADS; ++u) {
        const int e = e0 + u * STEP;
        const long long q = q0 + e;
        ok[u] = e < SEQ_CHUNK && q < n;
        v[u] = -0.0;
        if (ok[u]) {
          const int jq = (int)(q / nx);
          const int i = 1 + (int)(q - (long long)jq * nx);
          const int j = ja + jq;
          const size_t o = at(g, j, i);
          v[u] = (mode == 0) ? a[o] : 0.5 * (a[o] * a[o] + b[o] * b[o]);
          ok[u] = is_fluid(c, nx, g.ny, j, i);
        }
      }
#pragma unroll
      for (int u = 0; u < SEQ_LOADS; ++u) {
        const int e = e0 + u * STEP;
        if (e < SEQ_CHUNK) dst[e] = ok[u] ? v[u] : -0.0;
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
      const int len = (int)(left < SEQ_CHUNK ? (left + SEQ_BLOCK - 1) / SEQ_BLOCK * SEQ_BLOCK : SEQ_CHUNK);
      // blocks of SEQ_BLOCK terms, each fully unrolled: batch b+1's loads are
      // issued before batch b's adds (the asm ties the adds to the point after
      // the loads, and the loads may not sink below it), and the two register
      // batches alternate by name - no loop-carried copies, which a rolled
      // loop's registers cost (v_mov per term)
      for (int k0 = 0; k0 < len; k0 += SEQ_BLOCK) {
        double d[2][SEQ_BATCH];
#pragma unroll
        for (int u = 0; u < SEQ_BATCH; ++u) d[0][u] = src[k0 + u];
#pragma unroll
        for (int bb = 0; bb < SEQ_BLOCK / SEQ_BATCH; ++bb) {
          if (bb + 1 < SEQ_BLOCK / SEQ_BATCH) {
#pragma unroll
            for (int u = 0; u < SEQ_BATCH; ++u) d[(bb + 1) & 1][u] = src[k0 + (bb + 1) * SEQ_BATCH + u];
          }
          asm volatile("" : "+v"(s)::"memory");
#pragma unroll
          for (int u = 0; u < SEQ_BATCH; ++u) s += d[bb & 1][u];
        }
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
