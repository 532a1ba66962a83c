// resident.hpp — the SOR solve as ONE persistent launch whose workgroups keep
// their tile of p (and the source) on chip for the whole solve: grids of up to
// a few million cells (BASELINE configs[1] cavity 1024^2, configs[2] channel
// 4096x512), in red-black order and in the reference's own lexicographic
// order (resident.hip LEX: the skewed half-sweep schedule of lexw.hpp).
//
// Why: at these sizes the per-launch designs are bound by fill, not by HBM.
// The wave march gives each band 8-16 rows against a 15-19-row pipeline; the
// LDS tiles (tile.hip) reload and store their tile every 4 sweeps and run
// their sweeps latency- and barrier-bound out of LDS. Here the
// whole grid lives in the register files of the 256 CUs: nothing moves
// through HBM between sweeps except the tiles' edge bands.
//
// Layout: one workgroup of up to 8 waves per tile (at most one per CU, all
// co-resident). A tile owns res_tw = 112 (red-black) / 96 (reference order,
// cavity) / 104 (reference order, channel) columns x th rows (ghost rows / columns included at the grid's edges) and
// holds a region of 128 columns x (th + 2 res_halo) rows: lane l of every wave holds the column pair
// (c0 + 2l, c0 + 2l + 1), wave w the region rows w*RPW .. w*RPW + RPW - 1 of p
// in registers; the source as f*h^2 in registers (cavity, 8- or 10-row waves)
// or as f in LDS (channel: 14-row waves fit 4096x512's 102- / 110-row regions). A
// half-sweep updates one colour in place (its neighbours are the other
// colour): row neighbours within a lane's rows, column neighbours by DPP, the
// rows of the neighbouring waves through LDS (one barrier per half-sweep). The
// channel's ghost refreshes are cells of their own colour with copy rules.
//
// Groups: every res_ns sweeps the tiles exchange their res_halo-deep edge
// bands through global memory (write-through stores, one flag per tile and
// group; each tile waits for its <= 8 neighbours only): within a group the
// halo goes stale by one cell per half-sweep and never reaches the owned
// cells (res_halo = 2 res_ns), exactly as the fused march launches' halos.
// Red-black groups are 4 sweeps (its proof bounds grow 9x per sweep of a
// group), the reference order's 8 (cavity) / 6 (channel: deeper halos would
// not fit its regions in the waves' registers and LDS): the hand-off (~3 us
// a hop, the write-through stores' visibility) is paid every 8 / 6 sweeps
// instead of 4 for 1.2-1.4x the redundant halo work (1024^2: 2.53 -> 2.03 us
// per sweep).
//
// Stop rule, with no grid barrier (completion spreads one tile per group, so
// at group m every tile has finished group m - DIAM):
//  * red-black: proof mode - tiles prove "the reference goes
//    on" per iteration from black cells' max |p' - p|; an iteration no tile
//    proves ends the launch with code 2 at its group's first iteration k0:
//    the host replays to k0 from the intact input and goes on with the exact
//    launches (Solver::solve_resident);
//  * reference order: one sampled row per wave evaluates exact residuals (the
//    reference's operands) into per-iteration exceedance bits; an iteration
//    without one hands the solve to lexw.hpp (Solver::solve_resident_lex).
//
// Bits: every update is sor_update's operations on the same operands in the
// same order as the per-launch kernels and the oracle's restatements (the
// cavity's f*h^2 precomputed: the same rounding), so p is bit-identical.
#pragma once

#include "device.hpp"

namespace cfd {

#ifndef CFD_RES_NS_LEX
#define CFD_RES_NS_LEX 6
#endif
#ifndef CFD_RES_NS_LEX_CAV
#define CFD_RES_NS_LEX_CAV 8
#endif
constexpr int RES_NS_RB = 4;                      // sweeps per group, red-black
constexpr int RES_NS_LEX = CFD_RES_NS_LEX;        // sweeps per group, the reference's order (channel)
constexpr int RES_NS_LEX_CAV = CFD_RES_NS_LEX_CAV;  // ... (cavity)
__host__ __device__ constexpr int res_ns(bool open, bool lex) {
  return lex ? (open ? RES_NS_LEX : RES_NS_LEX_CAV) : RES_NS_RB;
}
__host__ __device__ constexpr int res_halo(bool open, bool lex) { return 2 * res_ns(open, lex); }  // halo cells per side
__host__ __device__ constexpr int res_tw(bool open, bool lex) { return 128 - 2 * res_halo(open, lex); }  // owned columns
constexpr int RES_MAXW = 8;                  // waves per workgroup, at most (2 per SIMD: 256 VGPRs each)
constexpr int RES_LAG = 2;                   // group g is checked at the start of group g + RES_LAG
constexpr int RES_REPLAY = 1;                // flags: no stop test (the host replays to a known count)

struct ResPlan {
  int ctiles, rtiles;  // column tiles (res_tw owned columns) x row tiles (th owned rows)
  int th;              // owned rows per tile (even)
  int lo, hi;          // owned rows [lo, hi) of the strip (ghost rows included; lo even)
  int waves;           // waves per workgroup (region rows th + 2 res_halo, rpw per wave)
  int rpw;             // region rows per wave (template parameter of the kernel)
};

// Device state of one resident solve (zeroed before every launch: the flags
// count groups of this launch only).
struct ResCtl {
  double* xa;           // edge bands of even groups (a full field, owned cells of the bands only)
  double* xb;           // ... of odd groups
  unsigned* flags;      // [tiles] groups each tile has completed and published
  unsigned* proven;     // [K + 1] 1: some tile proved iteration k goes on
  int* status;          // [0] 0 cap reached, 1 stop at [1] (only k = 0 here), 2 iteration [1] + 1 left
                        // open (fallback); [2] != 0: a wait timed out (never expected)
  const double* tol;    // [0] tolerance, [1] initial residual, [2] max|f| (tol_kernel)
  int K;                // sweeps to run (the cap, or the replayed count)
  int check_every;      // the reference tests every iteration (1)
  // the reference's order (LEX): exceedance bits, 8 shards of bwords words;
  // iteration k is bit k + koff (koff covers the cells that have not started)
  unsigned long long* bits;
  int bwords, koff;
};

// Tiling of a strip's owned rows [lo, hi) into at most max_tiles tiles, or
// ctiles = 0 if the grid does not fit (the solver keeps the per-launch kernels)
ResPlan res_plan(int nx, int lo, int hi, int max_tiles, bool open, bool lex);
// the channel's ghost refresh of a final field (red-black resident solve)
void res_refresh(const Geo& g, double* p, hipStream_t st);
constexpr int RES_RPW_OPEN = 14;  // rows per wave of the channel's larger tiles (reference order)
__host__ __device__ inline int res_groups(int K) { return (K + RES_NS_RB - 1) / RES_NS_RB; }  // (red-black)
// unsigned words of flags + proofs + status, rounded to 16 B
inline size_t res_state_words(int tiles, int K) {
  const size_t n = (size_t)tiles + (size_t)K + 1 + 8;
  return (n + 3) / 4 * 4;
}
// tiles of plan rp that can be resident at once on n_cu CUs (occupancy of the
// kernel instance with its LDS; 0: no instance): the persistent launch's
// workgroups spin on each other, so a plan above this must not launch
int res_coresident_tiles(int case_id, bool lex, const ResPlan& rp, int n_cu);
// throws cfd::Error when the pair has no kernel instance
void res_launch(int case_id, bool lex, const Geo& g, const Coef& c, const double* pin, double* pout, const double* f,
                const ResCtl& R, const ResPlan& rp, int flags, hipStream_t st);
// LEX exceedance-bit words per shard for K iterations on an nx x ny grid, and the bit offset
inline int res_lex_koff(int nx, int ny) { return (nx + ny) / 2 + 192; }
inline int res_lex_words(int nx, int ny, int K) { return (res_lex_koff(nx, ny) + K + 256) / 64 + 2; }

}  // namespace cfd
