// seqsum.hip — sequential sums in the reference's loop order, bit for bit.
//
// The reference-order mode (ordering = CFD_ORDER_LEX) reproduces the
// reference's own sums: the channel's / step's source mean (channel-01.cpp:
// 620-628, backwards_step-01.cpp:843-866) once per timestep and the kinetic
// energy of the statistics (cavity-01.cpp:750-755). Each partial sum is
// rounded before the next term is added: s_{k+1} = RN(s_k + x_k). As one
// chain of dependent fp64 adds that costs 2.9 ns per term on MI355X
// (tools/add_chain.hip), 6.7 ms for the channel's 4096 x 512 terms.
//
// Binade-chunked evaluation (same bits, in parallel where it is provable).
// While s_k stays in one binade [2^(U+52), 2^(U+53)) of magnitude, with one
// sign, s_k = S_k * 2^U for an integer S_k, and when the exact s_k + x_k stays
// in that binade too its rounding is to the nearest multiple of 2^U:
//   RN(s_k + x_k) = (S_k + r_k) * 2^U,  r_k = nearest integer to x_k * 2^-U,
// independent of S_k - unless x_k * 2^-U = q + 1/2 exactly: then the tie goes
// to the even one of S_k + q, S_k + q + 1, so r_k = q + ((S_k + q) & 1) depends
// on the parity of S_k only. So a run of terms is an integer sum, kept as two
// records, one per parity of the incoming S (they differ only after a tie).
// The terms are cut into chunks of SQ_CH in loop order (one wave each):
//  1. seq_approx_kernel: each chunk's approximate sum (any order);
//  2. seq_units_kernel (one workgroup): the approximate running sum at each
//     chunk's start (start value + the sums before it) guesses its unit U;
//  3. seq_chunk_kernel: the chunk's r_k under that U give, per incoming
//     parity, R = sum r_k and the minimum / maximum of the chunk's integer
//     prefix sums (0 included); a term too large for the binade or a
//     non-finite one marks the chunk "serial";
//  4. seq_walk_kernel (one workgroup): the exact chain over chunks. The
//     records of the next (up to) 64 chunks of one unit are combined into
//     prefix records across a wave's lanes (an ordered scan: lane l holds
//     chunks k..k+l); each lane checks its prefix against the exact running
//     sum s: with S = s * 2^-U, it holds when |S| is in [2^52, 2^53) (s in
//     the guessed binade) and S + min, S + max both lie in [2^52 + 1,
//     2^53 - 1] (or its negative) - every rounded partial sum S_{k+1} then
//     lies there, so every exact s_k + x_k (within half a unit of it) lies in
//     the binade and rounds as above. The check is exact (the guess only has
//     to be right) and monotone in l, so the longest passing prefix is taken
//     as S + R in one step. A chunk whose own record fails (the first terms
//     from zero, a binade crossing, a wrong guess) runs as the plain chain:
//     its terms staged in LDS, wave 0 adds them one by one.
// On the open cases' sources (scripts/dbg/seqsum_study.py) the running sum
// keeps one sign and crosses ~15 binades: ~10 plain chunks per sum, the rest
// in a few dozen walk steps.
//
// A solid cell is the term -0.0, which leaves every sum unchanged
// (x + -0.0 == x, -0.0 + -0.0 == -0.0), as skipping it does, and is r = 0.
#include "seqsum.hpp"

namespace cfd {

namespace {

constexpr int SQ_CH = 512;                 // terms per chunk (one wave: 8 consecutive terms per lane)
constexpr int SQ_TPL = SQ_CH / 64;         // terms per lane
constexpr int SQ_THREADS = 256;            // 4 chunks per workgroup (approx, chunk kernels); walk
constexpr int SQ_SCAN = 1024;              // seq_units_kernel threads
constexpr int SQ_BATCH = 32;               // terms the serial adder has in registers
constexpr int SQ_META_BATCH = SQ_THREADS;  // chunk records staged in LDS per walk batch
static_assert(SQ_CH % 64 == 0 && SQ_CH % SQ_BATCH == 0 && SQ_CH % SQ_THREADS == 0, "seqsum blocking");

struct Rec {
  long long r, lo, hi;  // sum of r_k, min / max of the prefix sums (0 included)
};
struct ChunkMeta {
  Rec e[2];    // per parity of the incoming integer sum
  int u;       // the guessed binade's unit exponent U
  int serial;  // 1: the chunk runs as the plain chain
};

// The terms in loop order: term q is cell (ja + q / nx, 1 + q % nx); a lane
// reads consecutive terms from one cursor (one division).
struct Terms {
  Geo g;
  Coef c;
  const double* a;
  const double* b;
  int mode, ja, jb;  // rows ja..jb
  struct Cur {
    int j, i;
  };
  __device__ __forceinline__ Cur cursor(unsigned q) const {
    const unsigned jq = q / (unsigned)g.nx;
    return Cur{ja + (int)jq, 1 + (int)(q - jq * (unsigned)g.nx)};
  }
  __device__ __forceinline__ double take(Cur& k) const {  // the term at k, then k advances
    double v = -0.0;
    if (k.j <= jb) {
      const size_t o = at(g, k.j, k.i);
      const double x = (mode == 0) ? a[o] : 0.5 * (a[o] * a[o] + b[o] * b[o]);
      v = is_fluid(c, g.nx, g.ny, k.j, k.i) ? x : -0.0;
    }
    if (++k.i > g.nx) {
      k.i = 1;
      ++k.j;
    }
    return v;
  }
};

// x then y: x's record p hands y the parity (p + x.r) & 1 (selects, no
// indexing: a private array indexed at run time would live in scratch)
__device__ __forceinline__ ChunkMeta meta_combine(const ChunkMeta& x, const ChunkMeta& y) {
  ChunkMeta z;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const Rec& a = x.e[p];
    const bool odd = ((p + a.r) & 1) != 0;
    const long long br = odd ? y.e[1].r : y.e[0].r;
    const long long blo = odd ? y.e[1].lo : y.e[0].lo;
    const long long bhi = odd ? y.e[1].hi : y.e[0].hi;
    z.e[p].lo = min(a.lo, a.r + blo);
    z.e[p].hi = max(a.hi, a.r + bhi);
    z.e[p].r = a.r + br;
  }
  z.u = x.u;
  z.serial = x.serial | y.serial;
  return z;
}

__device__ __forceinline__ ChunkMeta meta_shfl_up(const ChunkMeta& m, int off) {
  ChunkMeta y;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    y.e[p].r = __shfl_up(m.e[p].r, off, 64);
    y.e[p].lo = __shfl_up(m.e[p].lo, off, 64);
    y.e[p].hi = __shfl_up(m.e[p].hi, off, 64);
  }
  y.u = m.u;
  y.serial = __shfl_up(m.serial, off, 64);
  return y;
}

// ordered inclusive scan over a wave's lanes: lane l ends with lanes 0..l combined
__device__ __forceinline__ void wave_scan(ChunkMeta& m, int lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const ChunkMeta y = meta_shfl_up(m, off);
    if (lane >= off) m = meta_combine(y, m);
  }
}

__global__ __launch_bounds__(SQ_THREADS) void seq_approx_kernel(Terms tm, int nch, double* __restrict__ approx) {
  const int c = blockIdx.x * (SQ_THREADS / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (c >= nch) return;  // (wave-uniform)
  auto k = tm.cursor((unsigned)c * SQ_CH + lane * SQ_TPL);
  double v = 0.0;
#pragma unroll
  for (int e = 0; e < SQ_TPL; ++e) v += tm.take(k);
  v = wave_sum(v);
  if (lane == 0) approx[c] = v;
}

// units[c] = the unit exponent of the approximate running sum at chunk c's start
__global__ __launch_bounds__(SQ_SCAN) void seq_units_kernel(const double* __restrict__ approx, int nch,
                                                            const double* __restrict__ start, int accumulate,
                                                            int* __restrict__ units) {
  __shared__ double part[SQ_SCAN];
  const int t = threadIdx.x;
  const int per = (nch + SQ_SCAN - 1) / SQ_SCAN, c0 = t * per, c1 = min(nch, c0 + per);
  double v = 0.0;
  for (int c = c0; c < c1; ++c) v += approx[c];
  part[t] = v;
  __syncthreads();
  for (int off = 1; off < SQ_SCAN; off <<= 1) {  // inclusive scan of the thread sums (Hillis-Steele)
    const double y = t >= off ? part[t - off] : 0.0;
    __syncthreads();
    part[t] += y;
    __syncthreads();
  }
  double s = (accumulate ? start[0] : 0.0) + (t > 0 ? part[t - 1] : 0.0);
  for (int c = c0; c < c1; ++c) {
    int e = 0;
    (void)frexp(s, &e);  // |s| in [2^(e-1), 2^e): unit 2^(e-53)
    units[c] = e - 53;
    s += approx[c];
  }
}

__global__ __launch_bounds__(SQ_THREADS) void seq_chunk_kernel(Terms tm, int nch, const int* __restrict__ units,
                                                               ChunkMeta* __restrict__ meta) {
  const int c = blockIdx.x * (SQ_THREADS / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (c >= nch) return;  // (wave-uniform)
  const int u = units[c];
  ChunkMeta m{{{0, 0, 0}, {0, 0, 0}}, u, 0};
  auto k = tm.cursor((unsigned)c * SQ_CH + lane * SQ_TPL);
#pragma unroll
  for (int e = 0; e < SQ_TPL; ++e) {
    const double y = ldexp(tm.take(k), -u);
    long long r = 0, q = 0;
    bool tie = false;
    if (fabs(y) < 0x1p51) {  // (a larger term cannot keep the sum in one binade; NaN fails too)
      const double tr = trunc(y), fr = y - tr;  // exact
      tie = fabs(fr) == 0.5;
      q = (long long)tr - (fr < 0.0 ? 1 : 0);  // floor(y)
      r = (long long)tr + (fr > 0.5 ? 1 : 0) - (fr < -0.5 ? 1 : 0);
    } else {
      m.serial = 1;
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      Rec& a = m.e[p];
      a.r += tie ? q + ((p + a.r + q) & 1) : r;  // (the even neighbour of S + q)
      a.lo = min(a.lo, a.r);
      a.hi = max(a.hi, a.r);
    }
  }
  wave_scan(m, lane);  // lane 63: the chunk
  if (lane == 63) meta[c] = m;
}

// the exact check of record m at the running sum s; on success *out = s + m's terms
__device__ __forceinline__ bool meta_check(double s, const ChunkMeta& m, double* out) {
  if (m.serial) return false;
  const double S = ldexp(s, -m.u);
  const double A = fabs(S);
  if (!(A >= 0x1p52 && A < 0x1p53)) return false;  // (also: zero, non-finite)
  const long long Si = (long long)S;                 // exact: s is a multiple of 2^U
  const bool odd = (Si & 1) != 0;
  const long long er = odd ? m.e[1].r : m.e[0].r;
  const long long lo = Si + (odd ? m.e[1].lo : m.e[0].lo), hi = Si + (odd ? m.e[1].hi : m.e[0].hi);
  constexpr long long L = (1LL << 52) + 1, H = (1LL << 53) - 1;
  const bool ok = (Si > 0) ? (lo >= L && hi <= H) : (hi <= -L && lo >= -H);
  *out = ldexp((double)(Si + er), m.u);  // |S + R| < 2^53 when ok: exact
  return ok;
}

__global__ __launch_bounds__(SQ_THREADS) void seq_walk_kernel(Terms tm, const ChunkMeta* __restrict__ meta,
                                                              int nch, double* __restrict__ out, int accumulate,
                                                              int* __restrict__ serial_count) {
  __shared__ double buf[SQ_CH];
  __shared__ ChunkMeta mb[SQ_META_BATCH];
  __shared__ double sh_s;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  double s = accumulate ? out[0] : 0.0;  // the same value in every thread: uniform control flow
  int nser = 0;
#ifdef CFD_SEQ_STAMPS  // diagnostic build: wall-clock ticks (100 MHz) per phase into serial_count[1..5]
  long long ts[5] = {0, 0, 0, 0, 0}, tq = wall_clock64();
#define SEQ_STAMP(x) do { const long long tn = wall_clock64(); ts[x] += tn - tq; tq = tn; } while (0)
#else
#define SEQ_STAMP(x) do {} while (0)
#endif
  for (int c0 = 0; c0 < nch; c0 += SQ_META_BATCH) {
    __syncthreads();
    if (c0 + t < nch) mb[t] = meta[c0 + t];
    __syncthreads();
    SEQ_STAMP(0);
    const int cn = min(SQ_META_BATCH, nch - c0);
    for (int k = 0; k < cn;) {
      // prefix records of the chunks k.. of chunk k's unit (every wave
      // computes the same); the longest prefix that passes the check is taken
      const int u0 = mb[k].u;
      ChunkMeta x = mb[min(k + lane, cn - 1)];
      const bool fit = k + lane < cn && x.u == u0;
      const unsigned long long run_bits = __ballot(fit);
      const int run = (~run_bits == 0ull) ? 64 : __builtin_ctzll(~run_bits);
      if (lane >= run) x = ChunkMeta{{{0, 0, 0}, {0, 0, 0}}, u0, 0};
      wave_scan(x, lane);
      double sl;
      const bool ok = meta_check(s, x, &sl) && lane < run;
      const unsigned long long ok_bits = __ballot(ok);
      const int take = (~ok_bits == 0ull) ? 64 : __builtin_ctzll(~ok_bits);
      if (take > 0) {
        s = __shfl(sl, take - 1, 64);
        k += take;
        SEQ_STAMP(1);
        continue;
      }
      SEQ_STAMP(2);
      // the plain chain over chunk k
      ++nser;
      auto cur = tm.cursor((unsigned)(c0 + k) * SQ_CH + t * (SQ_CH / SQ_THREADS));
#pragma unroll
      for (int e = 0; e < SQ_CH / SQ_THREADS; ++e) buf[t * (SQ_CH / SQ_THREADS) + e] = tm.take(cur);
      __syncthreads();
      SEQ_STAMP(3);
      if (w == 0) {
        // every lane adds the same terms (broadcast reads), in order; batch
        // b+1's loads are issued before batch b's adds (the asm ties the adds
        // after the loads)
        double d[2][SQ_BATCH];
#pragma unroll
        for (int v = 0; v < SQ_BATCH; ++v) d[0][v] = buf[v];
#pragma unroll
        for (int bb = 0; bb < SQ_CH / SQ_BATCH; ++bb) {
          if (bb + 1 < SQ_CH / SQ_BATCH) {
#pragma unroll
            for (int v = 0; v < SQ_BATCH; ++v) d[(bb + 1) & 1][v] = buf[(bb + 1) * SQ_BATCH + v];
          }
          asm volatile("" : "+v"(s)::"memory");
#pragma unroll
          for (int v = 0; v < SQ_BATCH; ++v) s += d[bb & 1][v];
        }
        if (t == 0) sh_s = s;
      }
      __syncthreads();
      s = sh_s;
      ++k;
      SEQ_STAMP(4);
    }
  }
  if (t == 0) {
    out[0] = s;
    if (serial_count) serial_count[0] += nser;
#ifdef CFD_SEQ_STAMPS
    if (serial_count)
      for (int x = 0; x < 5; ++x) serial_count[1 + x] += (int)ts[x];
#endif
  }
}

}  // namespace

size_t seq_sum_workspace(long long n_terms) {
  const long long nch = (n_terms + SQ_CH - 1) / SQ_CH;
  return (size_t)nch * (sizeof(ChunkMeta) + sizeof(double) + sizeof(int)) + 64;
}

long long seq_sum_launch(const Geo& g, const Coef& c, const double* a, const double* b, int mode, double* out,
                         int accumulate, void* ws, size_t ws_bytes, int* serial_count, hipStream_t st) {
  const int ja = max(g.j0, 1), jb = min(g.j1, g.ny);
  const long long n = (long long)max(0, jb - ja + 1) * g.nx;
  const long long nch = (n + SQ_CH - 1) / SQ_CH;
  if (seq_sum_workspace(n) > ws_bytes) throw std::runtime_error("seq_sum: workspace too small");
  if (n + SQ_CH >= (1LL << 31)) throw std::runtime_error("seq_sum: too many terms in one strip");
  if (nch == 0) {
    if (!accumulate && hipMemsetAsync(out, 0, sizeof(double), st) != hipSuccess)
      throw std::runtime_error("seq_sum: hipMemsetAsync failed");
    return 0;
  }
  Terms tm{g, c, a, b, mode, ja, jb};
  auto* meta = reinterpret_cast<ChunkMeta*>(ws);  // (8-byte fields first)
  auto* approx = reinterpret_cast<double*>(meta + nch);
  auto* units = reinterpret_cast<int*>(approx + nch);
  const unsigned blocks = (unsigned)((nch + SQ_THREADS / 64 - 1) / (SQ_THREADS / 64));
  seq_approx_kernel<<<blocks, SQ_THREADS, 0, st>>>(tm, (int)nch, approx);
  seq_units_kernel<<<1, SQ_SCAN, 0, st>>>(approx, (int)nch, out, accumulate, units);
  seq_chunk_kernel<<<blocks, SQ_THREADS, 0, st>>>(tm, (int)nch, units, meta);
  seq_walk_kernel<<<1, SQ_THREADS, 0, st>>>(tm, meta, (int)nch, out, accumulate, serial_count);
  return nch;
}

}  // namespace cfd
