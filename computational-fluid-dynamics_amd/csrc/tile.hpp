// tile.hpp — red-black SOR launches for grids of a few million cells: each
// workgroup holds one tile of p in LDS and runs several whole sweeps on it.
//
// At 4096x512 (BASELINE configs[2]) or 1024^2 (configs[1]) the fused march
// launches (kernels.hpp poisson_multi_kernel) are bound by their pipeline
// fill, not by HBM: a resident round of 2048 waves gives each band ~8-10 rows
// against a 15-19-row fill, one dependent row step at a time.
// Here the grid is cut into at most one resident round of tiles, one 16-wave
// workgroup per CU. A workgroup loads its tile plus TILE_H cells of halo on
// every side (clamped to the stored strip) into LDS once, then runs `nsw`
// red-black iterations of the reference's SOR on it — red half-sweep | black
// half-sweep | [open cases: ghost / solid refresh] | max-norm residual, with
// a workgroup barrier between phases — and stores its owned cells once.
// The halo ring goes stale by one cell per dependent phase (red, black,
// refresh of a solid from its neighbour), never reaching the owned cells
// within the sweeps of one launch: 2 per sweep + the residual's 1 (cavity,
// channel), 3 per sweep + 1 for the step (its solids copy a neighbour after
// each sweep) - TILE_H = 10 covers 4 sweeps (3 for the step).
//
// Every cell sees the same operands in the same order as in the march
// kernels and the oracle's red-black restatement (sor_update, refresh_value,
// residual_abs of kernels.hpp), so p and every residual are bit-identical to
// them. Loads: p_in once (with the halos: 1.2-1.5x of the owned cells, mostly
// L2 hits), f once per launch into registers (each wave keeps the source of
// its rows for all sweeps); stores: p_out once.
//
// Layout in LDS: region row r (global row y0 - TILE_H + r) is 64 column pairs
// (128 columns: global x0 - TILE_H .. x0 + 117), lane l of a wave owns the
// pair (2l, 2l+1); wave w handles region rows w, w + 16, ...
#pragma once

#include "device.hpp"

namespace cfd {

constexpr int TILE_H = 10;               // halo cells per side (even: pairs stay 16-B aligned)
constexpr int TILE_W = 128 - 2 * TILE_H;  // owned columns per tile (108)
#ifndef CFD_TILE_WAVES
#define CFD_TILE_WAVES 16
#endif
constexpr int TILE_WAVES = CFD_TILE_WAVES;  // waves per workgroup (16: 1024 threads), one workgroup per CU
constexpr int TILE_ROWS = 128;              // region rows, at most (128 KiB of LDS)
constexpr int TILE_RPW = TILE_ROWS / TILE_WAVES;  // region rows per wave, at most
constexpr int TILE_MAX_TH = TILE_ROWS - 2 * TILE_H;  // owned rows per tile, at most
constexpr int TILE_ROWS_LDS = TILE_MAX_TH + 2 * TILE_H;  // region rows in LDS

struct TilePlan {
  int ctiles, rtiles;  // column tiles (TILE_W owned columns) x row tiles (th owned rows)
  int th;              // owned rows per tile
  int lo, hi;          // owned rows [lo, hi) of the strip (incl. physical ghost rows)
};

// sweeps one tile launch may run: each sweep costs the halo 2 cells (3 for the
// step's solid refresh), the last residual one more
__host__ __device__ constexpr int tile_max_sweeps(int case_id) {
  return case_id == BACKSTEP ? (TILE_H - 1) / 3 : (TILE_H - 1) / 2;
}

// Tiling of a strip's owned rows [lo, hi) into at most `max_tiles` tiles
// (0 tiles: the strip needs more, the caller keeps the march launches).
TilePlan tile_plan(int nx, int lo, int hi, int max_tiles);

// One launch: iterations k .. k+nsw-1 (nsw <= tile_max_sweeps), testing
// [ka, kb] first like poisson_multi_kernel (flags bit 2: no test, a replay;
// bit 1: XCD-aware tile order; bit 7: the tested window holds proof ratios).
// proof: the ring slots get proof ratios instead of residuals (no residual
// phase; DESIGN.md §2, tile.hip tile_proof_ratio).
void tile_launch(int case_id, bool proof, const Geo& g, const Coef& c, const double* pin, double* pout, const double* f,
                 const PoissonCtl& ctl, int k, int ka, int kb, int nsw, const TilePlan& tp, int flags,
                 hipStream_t st);

}  // namespace cfd
