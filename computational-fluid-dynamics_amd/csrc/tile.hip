// tile.hip — the LDS-tile red-black SOR launch (tile.hpp has the design).
// Own translation unit: device.hpp only (no kernels shared with solver.hip).
#include <algorithm>

#include "tile.hpp"

namespace cfd {

// refresh (open cases): does the tile's region hold a ghost row / column or a
// solid cell next to fluid? (tile-uniform)
__device__ __forceinline__ bool tile_refreshes(const Coef& c, int nx, int ny, int gy0, int rh, int gx0) {
  const int gy1 = gy0 + rh - 1, gx1 = gx0 + 127;
  if (gy0 <= 0 || gy1 >= ny + 1 || gx0 <= 0 || gx1 >= nx + 1) return true;
  // backwards step: solid block i <= step_i, j > inlet_jmax (its boundary cells)
  return c.case_id == BACKSTEP && gx0 <= c.step_i + 1 && gy1 >= c.inlet_jmax;
}

// rows one after another within a wave (the 16 waves of the workgroup hide
// the LDS latency): without it the unrolled row loops hoist every row's loads
// and spill
#ifndef CFD_TILE_FENCE
#define CFD_TILE_FENCE 1
#endif
// rows per scheduling group (CFD_TILE_FENCE_ROWS): the rows of a group are
// scheduled together (their LDS loads issued before their arithmetic: two
// independent chains in flight per wave)
#ifndef CFD_TILE_FENCE_ROWS
#define CFD_TILE_FENCE_ROWS 1
#endif
#if CFD_TILE_FENCE
#define TILE_ROW_FENCE(q)                                                    \
  do {                                                                       \
    if (((q) + 1) % CFD_TILE_FENCE_ROWS == 0) __builtin_amdgcn_sched_barrier(0); \
  } while (0)
#else
#define TILE_ROW_FENCE(q) ((void)0)
#endif
// 1: each wave owns a contiguous band of region rows and marches it, rows
// j-1 and j kept in registers (one LDS row load per row and phase instead of
// three); 0: waves take every 16th row
// (measured: interleaved rows 0.3-0.5 us per sweep faster - the band's
// sequential chain of LDS loads is latency-bound)
#ifndef CFD_TILE_BAND
#define CFD_TILE_BAND 0
#endif
// diagnostic build only (CFD_TILE_STAMPS=1, never the product library): each
// wave sums the shader-clock cycles of its phases (load, red, red barrier,
// black, black barrier, refresh, residual, store) over the launch's sweeps
// into a buffer of its own, read back by cfd_tile_stamps (shares, not times:
// the stamps' waits forbid overlaps the real kernel has)
#ifndef CFD_TILE_STAMPS
#define CFD_TILE_STAMPS 0
#endif
// 1: the cavity's sweeps skip the region rows outside the dependency cone of
// the owned rows (the open cases' refresh widens their cone: all rows)
#ifndef CFD_TILE_CONE
#define CFD_TILE_CONE 1
#endif
#if CFD_TILE_STAMPS
constexpr int STAMP_SEGS = 8;
__device__ unsigned long long tile_stamp_buf[1024 * TILE_WAVES * STAMP_SEGS];
#define TILE_STAMP(seg)                                                                     \
  do {                                                                                      \
    unsigned long long t_;                                                                  \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");              \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    st_acc[seg] += t_ - st_last;                                                            \
    st_last = t_;                                                                           \
  } while (0)
#else
#define TILE_STAMP(seg) ((void)0)
#endif

template <int CASE, bool PROOF>
__global__ __launch_bounds__(TILE_WAVES * 64) void poisson_tile_kernel(Geo g, Coef c, const double* __restrict__ pin,
                                                                        double* __restrict__ pout,
                                                                        const double* __restrict__ f, PoissonCtl ctl,
                                                                        int k, int ka, int kb, int nsw, TilePlan tp,
                                                                        int flags) {
  __shared__ double2 P[TILE_ROWS_LDS * 64];
  __shared__ double wred[TILE_WAVES];
  __shared__ int go;
  __shared__ double pinw[TILE_WAVES];  // proof mode: max |p_in| per wave
  double* Pd = reinterpret_cast<double*>(P);
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#if CFD_TILE_STAMPS
  unsigned long long st_acc[STAMP_SEGS] = {}, st_last;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_last)::"memory");
#endif

  const int nblk = (int)gridDim.x;
  const int L8 = (nblk / 8) * 8;
  const int bl = (int)blockIdx.x;
  // XCD-aware: consecutive tiles (neighbours along a row band) on one XCD
  const int tile = ((flags & 2) && bl < L8) ? (bl % 8) * (nblk / 8) + bl / 8 : bl;
  if (tile >= tp.ctiles * tp.rtiles) return;  // (whole workgroup)
  const int ct = tile % tp.ctiles, rt = tile / tp.ctiles;
  const int nx = g.nx, ny = g.ny;
  const int x0 = ct * TILE_W;
  const int y0 = tp.lo + rt * tp.th;
  const int y1 = min(y0 + tp.th, tp.hi);
  const int RH = (y1 - y0) + 2 * TILE_H;  // region rows (<= TILE_ROWS_LDS: host plan)
  const int gy0 = y0 - TILE_H;            // global row of region row 0
  const int gx = x0 - TILE_H + 2 * lane;  // this lane's columns gx (slot a), gx + 1 (slot b); gx even
  const int rmin = max(g.row_lo, 0), rmax = min(g.row_lo + g.nrows - 1, ny + 1);
  const int gxc = min(max(gx, 0), g.pitch - 2);
  constexpr bool BAND = CFD_TILE_BAND != 0;
  // this wave's region rows: row(q) for q < TILE_RPW while row(q) < rend
  const int RB = (RH + TILE_WAVES - 1) / TILE_WAVES;  // band height (<= TILE_RPW)
  const int r0 = BAND ? w * RB : w;
  const int rend = BAND ? min(r0 + RB, RH) : RH;
  auto row = [&](int q) { return BAND ? r0 + q : w + TILE_WAVES * q; };
  // the same rows from a base made opaque at the start of each phase: the
  // row-uniform conditions below are then recomputed per phase in SALU
  // instead of being hoisted out of the sweep loop as live SGPR masks (8 rows
  // x 2 colours of them spilled to VGPR lanes: v_readlane / v_writelane,
  // i.e. VALU work in every row)
  auto phase_rows = [&]() {
    int b = BAND ? r0 : w;
    asm volatile("" : "+s"(b));
    return b;
  };
  auto prow_q = [&](int b, int q) { return BAND ? b + q : b + TILE_WAVES * q; };
  // interleaved rows: row r's C / S / N, the row clamped into the region
  // (rows 0 and RH-1 are read, never updated). (Issuing each row's loads one
  // row ahead does not survive compilation: the optimiser sinks the current
  // row's loads into its branch, behind the next row's, and waits for both.)
  auto ld3 = [&](int r, double2& C, double2& S, double2& N) {
    const int rc = min(max(r, 1), RH - 2);
    C = P[rc * 64 + lane];
    S = P[(rc - 1) * 64 + lane];
    N = P[(rc + 1) * 64 + lane];
  };

  // p_in into LDS, f of this wave's rows into registers (rows / columns
  // clamped to stored memory: clamped cells lie outside the grid and are
  // never updated, refreshed or stored)
  double2 F[TILE_RPW];
  double pm = 0.0;  // proof mode: max |p_in| over the region (every cone of an owned cell lies in it)
  // every load first (addresses clamped, so no branch splits them: all of a
  // wave's rows are in flight at once), then the convergence test (its
  // latency overlaps the loads), then the LDS writes
  double2 V[TILE_RPW];
#pragma unroll
  for (int q = 0; q < TILE_RPW; ++q) {
    const int r = min(row(q), RH - 1);
    const int gyc = min(max(gy0 + r, rmin), rmax);
    const size_t o = (size_t)(gyc - g.row_lo) * (size_t)g.pitch + (size_t)gxc;
    V[q] = *reinterpret_cast<const double2*>(pin + o);
    F[q] = *reinterpret_cast<const double2*>(f + o);
  }
  // convergence test of the iterations [ka, kb] (flags bit 2: none, a replay),
  // decided by one wave for the whole workgroup (its barriers need all waves)
  if (w == 0) {
    const bool on = (flags & 4) || window_go_on(ctl, ka, kb, lane, blockIdx.x == 0, (flags & 128) != 0);
    if (lane == 0) go = on ? 1 : 0;
    if (on && blockIdx.x == 0 && lane < RES_SHARDS) {
      // the next launch's residual slots (as poisson_multi_kernel: RING_AHEAD)
#pragma unroll
      for (int q = 0; q < RING_AHEAD; ++q)
        ctl.ring[(size_t)((k + nsw + q) & (RING - 1)) * RES_SHARDS * SHARD_STRIDE + lane * SHARD_STRIDE] = 0.0;
    }
  }
#pragma unroll
  for (int q = 0; q < TILE_RPW; ++q) {
    const int r = row(q);
    if (r < rend) {
      P[r * 64 + lane] = V[q];
      if (PROOF) pm = fmax(pm, fmax(fabs(V[q].x), fabs(V[q].y)));
    }
  }
  if (PROOF) {
    pm = wave_max(pm);
    if (lane == 0) pinw[w] = pm;
  }
  __syncthreads();  // (also: the LDS tile written)
  if (!go) return;
  TILE_STAMP(0);

  const bool refr = CASE != CAVITY && tile_refreshes(c, nx, ny, gy0, RH, x0 - TILE_H);
  // lane constants of the two columns (slot a: gx, slot b: gx + 1): updated
  // (grid column, not the region's edge), owned (residual), the step's block
  // columns; the cavity's indicators as multipliers and omega / neighbour
  // count below / at the top row (cav_edge_sor: sor_update<CAVITY>'s operands)
  const bool upd_a = lane > 0 && gx >= 1 && gx <= nx;
  const bool upd_b = lane < 63 && gx + 1 >= 1 && gx + 1 <= nx;
  const bool own_a = 2 * lane >= TILE_H && 2 * lane < TILE_H + TILE_W && gx >= 1 && gx <= nx;
  const bool own_b = 2 * lane + 1 >= TILE_H && 2 * lane + 1 < TILE_H + TILE_W && gx + 1 >= 1 && gx + 1 <= nx;
  const bool blk_a = CASE == BACKSTEP && gx <= c.step_i, blk_b = CASE == BACKSTEP && gx + 1 <= c.step_i;
  // proof mode: owned black cells whose four neighbours the sweep's refresh
  // leaves alone (cavity: 1 < i < nx, 1 <= j < ny; open cases: 2 <= i, j <=
  // n-1, and for the step none of them next to the solid block)
  const int plo = (CASE == CAVITY) ? 1 : 2;
  const bool prv_a = own_a && gx >= 2 && gx <= nx - 1, prv_b = own_b && gx + 1 >= 2 && gx + 1 <= nx - 1;
  const bool nb_a = CASE == BACKSTEP && gx <= c.step_i + 1, nb_b = CASE == BACKSTEP && gx + 1 <= c.step_i + 1;
  double ce_a = 1.0, cw_a = 1.0, ce_b = 1.0, cw_b = 1.0, om_a = 0.0, omt_a = 0.0, om_b = 0.0, omt_b = 0.0;
  if (CASE == CAVITY) {
    ce_a = gx < nx ? 1.0 : 0.0;
    cw_a = gx > 1 ? 1.0 : 0.0;
    ce_b = gx + 1 < nx ? 1.0 : 0.0;
    cw_b = gx + 1 > 1 ? 1.0 : 0.0;
    const int na = (gx < nx) + (gx > 1) + 1, nb = (gx + 1 < nx) + (gx + 1 > 1) + 1;  // + eps_n below the top
    // om_nc[n] by value (a run-time index into Coef would copy it to scratch)
    const double o1 = c.om_nc[1], o2 = c.om_nc[2], o3 = c.om_nc[3], o4 = c.om_nc[4];
    auto pick = [&](int n) { return n == 4 ? o4 : n == 3 ? o3 : n == 2 ? o2 : o1; };
    om_a = pick(na + 1);
    omt_a = pick(na);
    om_b = pick(nb + 1);
    omt_b = pick(nb);
  }

  for (int s = 0; s < nsw; ++s) {
    // (opaque per sweep: products of the sources are not hoisted out of the
    // sweep loop, where they would hold 2 registers each)
#pragma unroll
    for (int q = 0; q < TILE_RPW; ++q) asm volatile("" : "+v"(F[q].x), "+v"(F[q].y));
    double dmx = 0.0;  // proof mode: max |p' - p| of this wave's proving black cells
    // red (i + j even), then black half-sweep (sor_update: cavity-01.cpp:643-654,
    // channel-01.cpp:659-666, backwards_step-01.cpp:900-909). Slot a (column
    // gx, even) has the colour of its row's parity: the slot is wave-uniform.
#pragma unroll
    for (int col = 0; col < 2; ++col) {
      // band march: rows r-1 and r in registers (the colour updated here is
      // never a vertical neighbour's colour, so the pre-update copies serve)
      const double2 z2 = make_double2(0.0, 0.0);
      double2 Sv = z2, Cv = z2;
      if (BAND) {
        if (r0 >= 1 && r0 - 1 < RH) Sv = P[(r0 - 1) * 64 + lane];
        if (r0 < RH) Cv = P[r0 * 64 + lane];
      }
      const int rb = phase_rows();
      // cavity: region rows inside the dependency cone of what the launch
      // evaluates (owned rows TILE_H .. RH-TILE_H-1 after nsw sweeps; black of
      // sweep s reaches 2(nsw-1-s) rows beyond them, red one more, exact
      // residuals read one row further): the rows outside never feed an owned
      // cell, a proving cell or a residual (same bits, fewer row updates)
      const int dist = 2 * (nsw - 1 - s) + (col == 0 ? 1 : 0) + (PROOF ? 0 : 1);
      const int clo = (CASE == CAVITY && CFD_TILE_CONE) ? max(1, TILE_H - dist) : 1;
      const int chi = (CASE == CAVITY && CFD_TILE_CONE) ? min(RH - 2, RH - 1 - TILE_H + dist) : RH - 2;
#pragma unroll
      for (int q = 0; q < TILE_RPW; ++q) {
        const int r = prow_q(rb, q);
        const int j = gy0 + r;
        if (!(r < rend)) break;
        double2 C = Cv, S = Sv, N = z2;
        if (BAND) {
          if (r + 1 < RH) N = P[(r + 1) * 64 + lane];
          Sv = Cv;
          Cv = N;
        } else {
          ld3(r, C, S, N);
        }
        // region rows with both neighbours in LDS, grid rows that are updated
        if (r >= clo && r <= chi && j >= 1 && j <= ny && j > rmin && j < rmax) {
          const bool open = CASE != BACKSTEP || j <= c.inlet_jmax;  // (row-uniform) the step's block rows: j > jmax
          const bool top = j == ny;
          // proof mode, black half-sweep: this row's cells prove (row-uniform part)
          const bool prow = PROOF && col == 1 && j >= plo && j <= ny - 1 && j >= y0 && j < y1 && j >= g.j0 &&
                            j <= g.j1;
          const bool pstep = CASE != BACKSTEP || j < c.inlet_jmax;  // below the block's lower neighbours
          if ((j & 1) == col) {
            const double W = dpp_from_left(C.y);
            const double nv = (CASE == CAVITY) ? cav_edge_sor(c, top, ce_a, cw_a, om_a, omt_a, C.x, W, C.y, S.x, N.x, F[q].x)
                                               : sor_interior<CASE>(c, C.x, W, C.y, S.x, N.x, F[q].x);
            if (upd_a && (open || !blk_a)) Pd[(r * 64 + lane) * 2] = nv;
            if (PROOF && prow && prv_a && (pstep || !nb_a)) dmx = fmax(dmx, fabs(nv - C.x));
          } else {
            const double E = dpp_from_right(C.x);
            const double nv = (CASE == CAVITY) ? cav_edge_sor(c, top, ce_b, cw_b, om_b, omt_b, C.y, C.x, E, S.y, N.y, F[q].y)
                                               : sor_interior<CASE>(c, C.y, C.x, E, S.y, N.y, F[q].y);
            if (upd_b && (open || !blk_b)) Pd[(r * 64 + lane) * 2 + 1] = nv;
            if (PROOF && prow && prv_b && (pstep || !nb_b)) dmx = fmax(dmx, fabs(nv - C.y));
          }
        }
        TILE_ROW_FENCE(q);
      }
      TILE_STAMP(1 + 2 * col);
      if (PROOF && col == 1) {
        dmx = wave_max(dmx);
        if (lane == 0) wred[w] = dmx;
      }
      __syncthreads();
      TILE_STAMP(2 + 2 * col);
    }
    if (PROOF && w == 0) {  // this sweep's ratio (wred: written before the barrier above, rewritten after the next)
      double v = lane < TILE_WAVES ? wred[lane] : 0.0, pv = lane < TILE_WAVES ? pinw[lane] : 0.0;
      v = wave_max(v);
      pv = wave_max(pv);
      double growth = 1.0;
      for (int q = 0; q < nsw; ++q) growth *= 9.0;
      const double ratio = proof_ratio_gen(c, ctl.tol[0], v, pv, ctl.tol[2], growth);
      if (lane == 0) {
        double* sl = ctl.ring + (size_t)((k + s) & (RING - 1)) * RES_SHARDS * SHARD_STRIDE;
        atomicMax(reinterpret_cast<unsigned long long*>(sl + (size_t)(tile % RES_SHARDS) * SHARD_STRIDE),
                  (unsigned long long)__double_as_longlong(ratio));
      }
    }
    // ghost / solid refresh from the swept field (channel-01.cpp:531-541,
    // backwards_step-01.cpp:685-740), as refresh_value: ghost rows / columns
    // first (from interior cells, none of which changes here), then the
    // step's solid cells next to fluid (from fluid cells only)
    if (CASE != CAVITY && refr) {
      const int rg = phase_rows();
#pragma unroll
      for (int q = 0; q < TILE_RPW; ++q) {
        const int r = prow_q(rg, q);
        const int j = gy0 + r;
        if (r < rend && r >= 1 && r <= RH - 2 && j >= 0 && j <= ny + 1) {
          double* pa = Pd + (r * 64 + lane) * 2;
          if (j == 0 || j == ny + 1) {  // ghost rows: p[0][i] = p[1][i], p[ny+1][i] = p[ny][i]
            const double2 V = P[(j == 0 ? r + 1 : r - 1) * 64 + lane];
            if (gx >= 1 && gx <= nx) pa[0] = V.x;
            if (gx + 1 >= 1 && gx + 1 <= nx) pa[1] = V.y;
          } else {  // ghost columns: p[j][0] = p[j][1] (slot a: column 0, so column 1 is slot b), p[j][nx+1] = 0
            if (gx == 0) pa[0] = pa[1];
            if (gx == nx + 1) pa[0] = 0.0;
            if (gx + 1 == nx + 1) pa[1] = 0.0;
          }
        }
      }
      __syncthreads();
      if (CASE == BACKSTEP) {
        const int rs = phase_rows();
#pragma unroll
        for (int q = 0; q < TILE_RPW; ++q) {
          const int r = prow_q(rs, q);
          const int j = gy0 + r;
          if (r < rend && r >= 1 && r <= RH - 2 && j > c.inlet_jmax && j <= ny) {  // rows of the solid block
            const double2 C = P[r * 64 + lane], S = P[(r - 1) * 64 + lane], N = P[(r + 1) * 64 + lane];
            const double W = dpp_from_left(C.y), E = dpp_from_right(C.x);
            double* pa = Pd + (r * 64 + lane) * 2;
            double out;
            if (lane > 0 && gx >= 1 && blk_a && refresh_value<CASE>(c, nx, ny, j, gx, C.x, W, C.y, S.x, N.x, out))
              pa[0] = out;
            if (lane < 63 && gx + 1 >= 1 && blk_b &&
                refresh_value<CASE>(c, nx, ny, j, gx + 1, C.y, C.x, E, S.y, N.y, out))
              pa[1] = out;
          }
        }
        __syncthreads();
      }
    }
    TILE_STAMP(5);
    // max-norm residual over the owned fluid cells (cavity-01.cpp:659-677,
    // channel-01.cpp:672-681, backwards_step-01.cpp:916-930) -> ring slot k+s
    if (PROOF) continue;
    double m = 0.0;
    const double2 z2 = make_double2(0.0, 0.0);
    double2 Sv = z2, Cv = z2;
    if (BAND) {
      if (r0 >= 1 && r0 - 1 < RH) Sv = P[(r0 - 1) * 64 + lane];
      if (r0 < RH) Cv = P[r0 * 64 + lane];
    }
    const int rr = phase_rows();
#pragma unroll
    for (int q = 0; q < TILE_RPW; ++q) {
      const int r = prow_q(rr, q);
      const int j = gy0 + r;
      if (!(r < rend)) break;
      double2 C = Cv, S = Sv, N = z2;
      const bool resrow = j >= y0 && j < y1 && j >= g.j0 && j <= g.j1;  // (owned rows: 1 <= r <= RH-2)
      if (BAND) {
        if (r + 1 < RH) N = P[(r + 1) * 64 + lane];
        Sv = Cv;
        Cv = N;
      } else {
        ld3(r, C, S, N);
      }
      if (resrow) {
        const bool open = CASE != BACKSTEP || j <= c.inlet_jmax;
        const double W = dpp_from_left(C.y), E = dpp_from_right(C.x);
        double ra, rb;
        if (CASE == CAVITY) {
          const bool top = j == ny;
          ra = cav_edge_res(c, top, ce_a, cw_a, C.x, W, C.y, S.x, N.x, F[q].x);
          rb = cav_edge_res(c, top, ce_b, cw_b, C.y, C.x, E, S.y, N.y, F[q].y);
        } else {
          ra = residual_interior<CASE>(c, C.x, W, C.y, S.x, N.x, F[q].x);
          rb = residual_interior<CASE>(c, C.y, C.x, E, S.y, N.y, F[q].y);
        }
        m = fmax(m, fmax((own_a && (open || !blk_a)) ? ra : 0.0, (own_b && (open || !blk_b)) ? rb : 0.0));
      }
      TILE_ROW_FENCE(q);
    }
    m = wave_max(m);
    if (lane == 0) wred[w] = m;
    __syncthreads();  // (also: the residual's reads before the next red writes)
    if (w == 0) {
      double v = lane < TILE_WAVES ? wred[lane] : 0.0;
      v = wave_max(v);
      if (lane == 0) {
        double* sl = ctl.ring + (size_t)((k + s) & (RING - 1)) * RES_SHARDS * SHARD_STRIDE;
        atomicMax(reinterpret_cast<unsigned long long*>(sl + (size_t)(tile % RES_SHARDS) * SHARD_STRIDE),
                  (unsigned long long)__double_as_longlong(v));
      }
    }
    TILE_STAMP(6);
  }
  // owned cells -> p_out (16-B pairs; columns up to the pitch)
  const bool st_lane = 2 * lane >= TILE_H && 2 * lane < TILE_H + TILE_W && gx >= 0 && gx + 1 < g.pitch;
#pragma unroll
  for (int q = 0; q < TILE_RPW; ++q) {
    const int r = row(q);
    const int j = gy0 + r;
    if (r < rend && j >= y0 && j < y1 && st_lane)
      *reinterpret_cast<double2*>(pout + (size_t)(j - g.row_lo) * (size_t)g.pitch + (size_t)gx) = P[r * 64 + lane];
  }
#if CFD_TILE_STAMPS
  __builtin_amdgcn_s_waitcnt(0);  // (the stores issued: their issue time, not their completion)
  TILE_STAMP(7);
  if (lane < STAMP_SEGS && bl < 1024) {
    unsigned long long v = 0;
#pragma unroll
    for (int q = 0; q < STAMP_SEGS; ++q) v = lane == q ? st_acc[q] : v;
    tile_stamp_buf[((size_t)bl * TILE_WAVES + w) * STAMP_SEGS + lane] = v;
  }
#endif
}

TilePlan tile_plan(int nx, int lo, int hi, int max_tiles) {
  TilePlan tp{};
  tp.lo = lo;
  tp.hi = hi;
  tp.ctiles = (nx + 2 + TILE_W - 1) / TILE_W;
  const int rows = hi - lo;
  const int rt_min = (rows + TILE_MAX_TH - 1) / TILE_MAX_TH;
  if (rows <= 0 || tp.ctiles * rt_min > max_tiles) return TilePlan{};  // does not fit: no tiles
  // as many row tiles as fit (short tiles: less time per sweep), at least 8 rows each
  int rt = std::max(rt_min, std::min(max_tiles / tp.ctiles, (rows + 7) / 8));
  tp.th = (rows + rt - 1) / rt;
  tp.rtiles = (rows + tp.th - 1) / tp.th;
  return tp;
}

void tile_launch(int case_id, bool proof, const Geo& g, const Coef& c, const double* pin, double* pout, const double* f,
                 const PoissonCtl& ctl, int k, int ka, int kb, int nsw, const TilePlan& tp, int flags,
                 hipStream_t st) {
  const int n = tp.ctiles * tp.rtiles;
  if (n <= 0) return;
  const dim3 grid(n), block(TILE_WAVES * 64);
#define CFD_TILE_LAUNCH(CASE, PR) \
  poisson_tile_kernel<CASE, PR><<<grid, block, 0, st>>>(g, c, pin, pout, f, ctl, k, ka, kb, nsw, tp, flags)
  if (case_id == CAVITY) {
    if (proof) CFD_TILE_LAUNCH(CAVITY, true); else CFD_TILE_LAUNCH(CAVITY, false);
  } else if (case_id == CHANNEL) {
    if (proof) CFD_TILE_LAUNCH(CHANNEL, true); else CFD_TILE_LAUNCH(CHANNEL, false);
  } else {
    if (proof) CFD_TILE_LAUNCH(BACKSTEP, true); else CFD_TILE_LAUNCH(BACKSTEP, false);
  }
#undef CFD_TILE_LAUNCH
}

#if CFD_TILE_STAMPS
// diagnostic build only: the last tile launch's per-wave phase cycle sums,
// [block][wave][segment] (1024 x TILE_WAVES x 8 values)
extern "C" int cfd_tile_stamps(unsigned long long* out, int n) {
  const int cap = 1024 * TILE_WAVES * STAMP_SEGS;
  if (n > cap) n = cap;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(tile_stamp_buf), (size_t)n * 8) == hipSuccess ? n : -1;
}
#endif

}  // namespace cfd
