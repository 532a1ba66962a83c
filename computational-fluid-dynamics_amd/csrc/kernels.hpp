// kernels.hpp — HIP kernels for the projection-method timestep on gfx950.
//
// Device-side restatement of the reference's per-timestep path
// (cavity-01.cpp, channel-01.cpp, backwards_step-01.cpp); every kernel cites
// the reference loop it replaces. Floating-point expressions keep the
// reference's operand order and the library is built with -ffp-contract=off,
// so the stencil kernels are bit-identical to the reference loops.
//
// Layout: each field of a strip is a row-major slab of
// `nrows` x `pitch` doubles; global cell (j, i) lives at
// (j - row_lo) * pitch + i. Row 0 / ny+1 and column 0 / nx+1 are the
// reference's ghost layers; a strip additionally stores HALO rows of its
// neighbours on each side.
#pragma once

#include "device.hpp"

namespace cfd {

// ------------------------------------------------------------------ BCs --

// cavity-01.cpp:523-543: moving lid + no-slip walls by ghost reflection.
__global__ void bc_cavity_kernel(Geo g, Coef c, double* __restrict__ u, double* __restrict__ v) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int nx = g.nx, ny = g.ny;
  if (t <= nx) {
    if (g.wj1 == ny + 1) u[at(g, ny + 1, t)] = 2.0 * c.u_ref - u[at(g, ny, t)];
    if (g.wj0 == 0) u[at(g, 0, t)] = -u[at(g, 1, t)];
  }
  const int vj_lo = g.wj0, vj_hi = g.wj1 < ny ? g.wj1 : ny;
  const int j = vj_lo + t;
  if (j <= vj_hi) {
    v[at(g, j, nx + 1)] = -v[at(g, j, nx)];
    v[at(g, j, 0)] = -v[at(g, j, 1)];
  }
}

// channel-01.cpp:513-529 / backwards_step-01.cpp:616-653, phases a-h merged:
// every write is computed from the pre-call state plus the in-call writes it
// depends on in the reference's order (u[1][0], u[ny][0], u[1][nx], u[ny][nx]).
__global__ void bc_open_kernel(Geo g, Coef c, double* __restrict__ u, double* __restrict__ v) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int nx = g.nx, ny = g.ny;
  const int jin = (c.case_id == BACKSTEP) ? c.inlet_jmax : ny;
  // column phases on owned rows: (a) u inlet, (b) v inlet, (c) u outlet, (d) v outlet
  const int j = g.wj0 + t;
  if (j <= g.wj1) {
    if (j >= 1 && j <= ny) {
      u[at(g, j, 0)] = (j <= jin) ? c.u_ref : 0.0;
      u[at(g, j, nx)] = u[at(g, j, nx - 1)];
    }
    if (j >= 0 && j <= ny) {
      v[at(g, j, 0)] = 0.0;
      // (d) on the boundary rows is done by the row phase's i == nx thread, which
      // must read v[j][nx] before (e)/(g) zero it (the reference order)
      const bool zrow = (j == 0 && g.wj0 == 0) || (j == ny && g.wj1 == ny + 1);
      if (!zrow) v[at(g, j, nx + 1)] = v[at(g, j, nx)];
    }
  }
  // row phases (e)-(h) on the physical boundary rows
  if (t <= nx) {
    const int i = t;
    if (g.wj0 == 0) {
      if (i == nx) v[at(g, 0, nx + 1)] = v[at(g, 0, nx)];
      if (i >= 1) v[at(g, 0, i)] = 0.0;
      // (f) u[0][i] = -u[1][i], with u[1][0] / u[1][nx] as set by (a) / (c)
      double u1;
      if (i == 0) u1 = (1 <= jin) ? c.u_ref : 0.0;
      else if (i == nx) u1 = u[at(g, 1, nx - 1)];
      else u1 = u[at(g, 1, i)];
      u[at(g, 0, i)] = -u1;
    }
    if (g.wj1 == ny + 1) {
      if (i == nx) v[at(g, ny, nx + 1)] = v[at(g, ny, nx)];
      if (i >= 1) v[at(g, ny, i)] = 0.0;
      double un;
      if (i == 0) un = (ny <= jin) ? c.u_ref : 0.0;
      else if (i == nx) un = u[at(g, ny, nx - 1)];
      else un = u[at(g, ny, i)];
      u[at(g, ny + 1, i)] = -un;
    }
  }
}

// backwards_step-01.cpp:654-682: zero the faces between solid and fluid
// cells, restated per face over the box that can border the solid block.
__global__ void bc_step_faces_kernel(Geo g, Coef c, double* __restrict__ u, double* __restrict__ v, int box_i1,
                                     int box_j0) {
  const int nx = g.nx, ny = g.ny;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // 0..box_i1
  const int j = box_j0 + blockIdx.y;
  if (i > box_i1 || j > g.wj1 || j < g.wj0) return;
  // u face (j, i), 1 <= j <= ny, 1 <= i <= nx-1 (interior faces the rule can touch)
  if (j >= 1 && j <= ny && i >= 1 && i <= nx - 1) {
    const bool a = is_fluid(c, nx, ny, j, i), b = is_fluid(c, nx, ny, j, i + 1);
    // solid (j,i) with fluid east neighbour, or solid (j,i+1) with fluid west neighbour
    if ((!a && b) || (!b && a)) u[at(g, j, i)] = 0.0;
  }
  // v face (j, i), 1 <= j <= ny-1
  if (j >= 1 && j <= ny - 1 && i >= 1 && i <= nx) {
    const bool a = is_fluid(c, nx, ny, j, i), b = is_fluid(c, nx, ny, j + 1, i);
    if ((!a && b) || (!b && a)) v[at(g, j, i)] = 0.0;
  }
}

// ------------------------------------------------------------ predictor --

// cavity-01.cpp:548-603 / channel-01.cpp:546-603 / backwards_step-01.cpp:745-820.
// Row march (like the SOR kernels): a wave owns 128 columns (2 per lane,
// 16-byte loads) and walks down a band of `th` rows keeping rows j-1, j, j+1
// of u and v in registers; column neighbours move between lanes by DPP. Each
// row costs one load of u and of v and the stores of u*, v* (32 B per cell plus
// 2 halo rows per band and 2 halo columns per 128). Output columns: 112 per
// wave, on 128-B lines (CFD_TENT_ALIGN, below). Same expressions in the same
// order as the reference loops, hence the same bits.
#ifndef CFD_TENT_ALIGN
// 1: tiles of 112 output columns starting on 128-B lines (lanes 4..59 store)
// 2: tiles of 128 output columns on 1-KB lines, every lane stores; the two
//    neighbour columns outside the tile come from one extra 8-byte load per
//    field and row (lane 0: column gi-1, lane 63: column gi+2) - measured
//    123 us at 4096^2 against 119.5 for 1 (the halo columns were L2 hits)
// 0: 126 output columns (lanes 1..63 / 0..62)
#define CFD_TENT_ALIGN 1
#endif
constexpr int TENT_TWC = CFD_TENT_ALIGN == 2 ? 128 : CFD_TENT_ALIGN ? 112 : 126;
#ifndef CFD_TENT_PD
#define CFD_TENT_PD 3  // rows of u and v in flight ahead of row j+1
#endif
#ifndef CFD_TENT_NT
#define CFD_TENT_NT 0  // nontemporal u*, v* stores
#endif
__global__ __launch_bounds__(256) void tentative_kernel(Geo g, Coef c, const double* __restrict__ u,
                                                        const double* __restrict__ v, double* __restrict__ us,
                                                        double* __restrict__ vs, int th, int ctiles) {
  const int lane = threadIdx.x & 63;
  const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int ctile = tile % ctiles, band = tile / ctiles;
  const int y0 = g.j0 + band * th, y1 = min(y0 + th, g.j1 + 1);
  if (y0 >= y1) return;
  const int nx = g.nx, ny = g.ny;
  const bool step = c.case_id == BACKSTEP;
  // this lane's columns gi (a), gi + 1 (b)
  const int gi = CFD_TENT_ALIGN == 1 ? ctile * TENT_TWC - 8 + 2 * lane : ctile * TENT_TWC + 2 * lane;
  const int gic = max(min(gi, g.pitch - 2), 0);     // (lanes past the row read a valid pair)
  const size_t P = (size_t)g.pitch;
  auto ld = [&](const double* base, int j) {
    return *reinterpret_cast<const double2*>(base + (size_t)(j - g.row_lo) * P + gic);
  };
  // output cells: a of lanes 1..63, b of lanes 0..62 (their row neighbours are in the wave)
  constexpr bool EDGEL = CFD_TENT_ALIGN == 2;
  const bool out_a = (EDGEL || (CFD_TENT_ALIGN ? lane >= 4 && lane <= 59 : lane >= 1)) && gi <= nx;
  const bool out_b = (EDGEL || (CFD_TENT_ALIGN ? lane >= 4 && lane <= 59 : lane <= 62)) && gi + 1 <= nx;
  // rows j+1 .. j+3 of u and v in flight (clamped to the strip's stored rows:
  // rows past y1 are never consumed)
  const int rlast = g.row_lo + g.nrows - 1;
  auto ldc = [&](const double* base, int j) { return ld(base, min(j, rlast)); };
  constexpr int PD = CFD_TENT_PD;
  double2 um = ld(u, y0 - 1), uc = ld(u, y0), vm = ld(v, y0 - 1), vc = ld(v, y0);
  double2 uq[PD], vq[PD];
#pragma unroll
  for (int q = 0; q < PD; ++q) {
    uq[q] = ldc(u, y0 + 1 + q);
    vq[q] = ldc(v, y0 + 1 + q);
  }
  // EDGEL: the column outside the tile next to lane 0 (gi - 1) / lane 63
  // (gi + 2); the other lanes read their own column (a line they load anyway)
  const int ge = EDGEL ? min(max(lane == 0 ? gi - 1 : lane == 63 ? gi + 2 : gi, 0), g.pitch - 1) : 0;
  auto lde = [&](const double* base, int j) { return base[(size_t)(min(j, rlast) - g.row_lo) * P + ge]; };
  double ue_c = 0.0, ve_m = 0.0, ve_c = 0.0, ueq[PD], veq[PD];
  if (EDGEL) {
    ue_c = lde(u, y0);
    ve_m = lde(v, y0 - 1);
    ve_c = lde(v, y0);
#pragma unroll
    for (int q = 0; q < PD; ++q) {
      ueq[q] = lde(u, y0 + 1 + q);
      veq[q] = lde(v, y0 + 1 + q);
    }
  }
  for (int j = y0; j < y1; ++j) {
    const double2 up = uq[0], vp = vq[0];
#pragma unroll
    for (int q = 0; q + 1 < PD; ++q) {
      uq[q] = uq[q + 1];
      vq[q] = vq[q + 1];
    }
    uq[PD - 1] = ldc(u, j + 1 + PD);
    vq[PD - 1] = ldc(v, j + 1 + PD);
    double uep = 0.0, vep = 0.0;
    if (EDGEL) {
      uep = ueq[0];
      vep = veq[0];
#pragma unroll
      for (int q = 0; q + 1 < PD; ++q) {
        ueq[q] = ueq[q + 1];
        veq[q] = veq[q + 1];
      }
      ueq[PD - 1] = lde(u, j + 1 + PD);
      veq[PD - 1] = lde(v, j + 1 + PD);
    }
    double uWa = dpp_from_left(uc.y), uEb = dpp_from_right(uc.x);
    double vEb = dpp_from_right(vc.x), vmEb = dpp_from_right(vm.x);
    double vWa = dpp_from_left(vc.y), upWa = dpp_from_left(up.y);
    if (EDGEL) {  // the tile's outer neighbours (same values, so the same bits)
      uWa = lane == 0 ? ue_c : uWa;
      vWa = lane == 0 ? ve_c : vWa;
      upWa = lane == 0 ? uep : upWa;
      uEb = lane == 63 ? ue_c : uEb;
      vEb = lane == 63 ? ve_c : vEb;
      vmEb = lane == 63 ? ve_m : vmEb;
    }
    double* usr = us + (size_t)(j - g.row_lo) * P;
    double* vsr = vs + (size_t)(j - g.row_lo) * P;
    double usv[2], vsv[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = gi + h;
      // u* on the face (j, i): cells 1..nx-1
      {
        const double cc = h == 0 ? uc.x : uc.y;
        const double uE = h == 0 ? uc.y : uEb, uW = h == 0 ? uWa : uc.x;
        const double uN = h == 0 ? up.x : up.y, uS = h == 0 ? um.x : um.y;
        const double diff = c.nu * ((uE - 2.0 * cc + uW) * c.idx2 + (uN - 2.0 * cc + uS) * c.idy2);
        const double ue = 0.5 * (cc + uE);
        const double uw = 0.5 * (uW + cc);
        const double cx = (ue * ue - uw * uw) * c.idx;
        const double vn = 0.5 * ((h == 0 ? vc.x : vc.y) + (h == 0 ? vc.y : vEb));
        const double vso = 0.5 * ((h == 0 ? vm.x : vm.y) + (h == 0 ? vm.y : vmEb));
        const double un = 0.5 * (uN + cc);
        const double uso = 0.5 * (uS + cc);
        const double cy = (vn * un - vso * uso) * c.idy;
        const double val = cc + c.dt * (diff - cx - cy);
        const bool valid = !step || is_fluid(c, nx, ny, j, i) || is_fluid(c, nx, ny, j, i + 1);
        usv[h] = valid ? val : 0.0;
      }
      // v* on the face (j, i): rows 1..ny-1
      {
        const double cc = h == 0 ? vc.x : vc.y;
        const double vE = h == 0 ? vc.y : vEb, vW = h == 0 ? vWa : vc.x;
        const double vN = h == 0 ? vp.x : vp.y, vS = h == 0 ? vm.x : vm.y;
        const double diff = c.nu * ((vE - 2.0 * cc + vW) * c.idx2 + (vN - 2.0 * cc + vS) * c.idy2);
        const double vn = 0.5 * (cc + vN);
        const double vso = 0.5 * (vS + cc);
        const double cy = (vn * vn - vso * vso) * c.idy;
        const double ue = 0.5 * ((h == 0 ? uc.x : uc.y) + (h == 0 ? up.x : up.y));
        const double uw = 0.5 * ((h == 0 ? uWa : uc.x) + (h == 0 ? upWa : up.x));
        const double ve = 0.5 * (cc + vE);
        const double vw = 0.5 * (vW + cc);
        const double cx = (ue * ve - uw * vw) * c.idx;
        const double val = cc + c.dt * (diff - cy - cx);
        const bool valid = !step || is_fluid(c, nx, ny, j, i) || is_fluid(c, nx, ny, j + 1, i);
        vsv[h] = valid ? val : 0.0;
      }
    }
    // 16-byte stores where both cells of the lane are written (coalesced rows),
    // single cells at the tile and grid edges
    const bool ua = out_a && gi >= 1 && gi <= nx - 1, ub = out_b && gi + 1 >= 1 && gi + 1 <= nx - 1;
    const bool va = out_a && gi >= 1 && j <= ny - 1, vb = out_b && gi + 1 <= nx && j <= ny - 1;
    typedef double d2v __attribute__((ext_vector_type(2)));
    if (ua && ub) {
      d2v w = {usv[0], usv[1]};
      if (CFD_TENT_NT) __builtin_nontemporal_store(w, reinterpret_cast<d2v*>(usr + gi));
      else *reinterpret_cast<d2v*>(usr + gi) = w;
    } else {
      if (ua) usr[gi] = usv[0];
      if (ub) usr[gi + 1] = usv[1];
    }
    if (va && vb) {
      d2v w = {vsv[0], vsv[1]};
      if (CFD_TENT_NT) __builtin_nontemporal_store(w, reinterpret_cast<d2v*>(vsr + gi));
      else *reinterpret_cast<d2v*>(vsr + gi) = w;
    } else {
      if (va) vsr[gi] = vsv[0];
      if (vb) vsr[gi + 1] = vsv[1];
    }
    um = uc; uc = up; vm = vc; vc = vp;
    if (EDGEL) {
      ue_c = uep;
      ve_m = ve_c;
      ve_c = vep;
    }
  }
}

// ------------------------------------------------------ Rayleigh-Benard --
// No reference solver (BASELINE configs[4]); restated in oracle/cfd_oracle.c
// (orc_temperature_bc, orc_thermal), bit-exact with it.

// Temperature ghosts: hot bottom / cold top by reflection (like the lid,
// cavity-01.cpp:523-529), adiabatic sides by copy; owned rows only.
__global__ void bc_temperature_kernel(Geo g, Coef c, double* __restrict__ T) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int nx = g.nx, ny = g.ny;
  const int i = t + 1;
  if (i <= nx) {
    if (g.wj0 == 0) T[at(g, 0, i)] = 2.0 * c.t_hot - T[at(g, 1, i)];
    if (g.wj1 == ny + 1) T[at(g, ny + 1, i)] = 2.0 * c.t_cold - T[at(g, ny, i)];
  }
  const int j = g.j0 + t;
  if (j <= g.j1) {
    T[at(g, j, 0)] = T[at(g, j, 1)];
    T[at(g, j, nx + 1)] = T[at(g, j, nx)];
  }
}

// One fused pass per cell: Boussinesq buoyancy on the v* face above it and
// the explicit central advection-diffusion update of T (face fluxes with the
// step's starting velocities). HBM-bound: reads T (5-point, rows reused via
// L2), u, v, v*; writes T2, v*.
__global__ __launch_bounds__(256) void thermal_kernel(Geo g, Coef c, const double* __restrict__ u,
                                                      const double* __restrict__ v, const double* __restrict__ T,
                                                      double* __restrict__ T2, double* __restrict__ vs) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j = g.j0 + blockIdx.y * 4 + (threadIdx.x >> 6);
  const int nx = g.nx, ny = g.ny;
  if (j > g.j1 || i < 1 || i > nx) return;
  const size_t o = at(g, j, i);
  const size_t P = (size_t)g.pitch;
  const double cc = T[o];
  const double tE = T[o + 1], tW = T[o - 1], tN = T[o + P], tS = T[o - P];
  if (j <= ny - 1) vs[o] = vs[o] + c.dt * (c.buoy * (0.5 * (cc + tN) - c.t_ref));
  const double diff = c.kappa * ((tE - 2.0 * cc + tW) * c.idx2 + (tN - 2.0 * cc + tS) * c.idy2);
  const double fe = u[o] * (0.5 * (cc + tE));
  const double fw = u[o - 1] * (0.5 * (tW + cc));
  const double fn = v[o] * (0.5 * (cc + tN));
  const double fs = v[o - P] * (0.5 * (tS + cc));
  T2[o] = cc + c.dt * (diff - (fe - fw) * c.idx - (fn - fs) * c.idy);
}

// --------------------------------------------------------------- source --

// cavity-01.cpp:622-630; channel-01.cpp:613-619 and backwards_step-01.cpp:830-841
// (f and, for the open cases, its per-block partial sum for the mean).
// Straight-line form: the address is formed once and the value selected, so
// no lane's store depends on which branch the wave took.
// The cavity's tolerance input max|f| (cavity-01.cpp:628) is reduced in the
// same pass into the srcmax shards (the open cases reduce it after the mean
// removal, subtract_mean_kernel): one read of f fewer per timestep.
__global__ __launch_bounds__(256) void source_kernel(Geo g, Coef c, const double* __restrict__ us,
                                                     const double* __restrict__ vs, double* __restrict__ f,
                                                     double* __restrict__ partials, double* __restrict__ srcmax) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j = g.j0 + blockIdx.y * 4 + (threadIdx.x >> 6);
  const int nx = g.nx, ny = g.ny;
  const bool inside = i >= 1 && i <= nx && j >= 1 && j <= ny && j <= g.j1;
  double val = 0.0;
  if (inside) {
    const size_t o = at(g, j, i);
    const double du = us[o] - us[o - 1];
    const double dv = vs[o] - vs[o - (size_t)g.pitch];
    const double cav = c.cav_src * (du * c.idx + dv * c.idx);
    const double opn = c.open_src * (du * c.idx + dv * c.idy);
    const bool fl = is_fluid(c, nx, ny, j, i);
    val = (c.case_id == CAVITY) ? cav : (fl ? opn : 0.0);
    f[o] = val;
  }
  if (c.case_id != CAVITY) {
    const double s = block_sum<256>(val);
    if (threadIdx.x == 0) partials[blockIdx.y * gridDim.x + blockIdx.x] = s;
  } else {
    block_max_to_shard<256>(fabs(val), srcmax, (blockIdx.y * gridDim.x + blockIdx.x) % RES_SHARDS);
  }
}

// Cavity source term + max|f| (cavity-01.cpp:622-630) on column pairs: a
// wave covers 128 columns of one row with 16-B loads and stores (u* of column
// i-1 by DPP; lane 0 loads it), a block 4 rows. Same expression per cell as
// source_kernel, hence the same bits; the open cases keep source_kernel (their
// mean's block-partial order).
__global__ __launch_bounds__(256) void cavity_source_kernel(Geo g, Coef c, const double* __restrict__ us,
                                                            const double* __restrict__ vs, double* __restrict__ f,
                                                            double* __restrict__ srcmax) {
  const int lane = threadIdx.x & 63;
  const int gi = blockIdx.x * 128 + 2 * lane;  // even: the pair (gi, gi + 1) is 16-B aligned (pitch % 16 == 0)
  const int j = max(g.j0, 1) + blockIdx.y * 4 + (threadIdx.x >> 6);
  const int nx = g.nx;
  double m = 0.0;
  if (j <= min(g.j1, g.ny) && gi <= nx) {  // (lanes past nx idle; a lane's left neighbour is active)
    const size_t o = at(g, j, gi), P = (size_t)g.pitch;
    const double2 uc = *reinterpret_cast<const double2*>(us + o);
    const double2 vc = *reinterpret_cast<const double2*>(vs + o);
    const double2 vm = *reinterpret_cast<const double2*>(vs + o - P);
    double uw = dpp_from_left(uc.y);
    if (lane == 0) uw = us[o - 1];  // (gi = 0: row j-1's last value, unused)
    const double dua = uc.x - uw, dub = uc.y - uc.x;
    const double dva = vc.x - vm.x, dvb = vc.y - vm.y;
    const double fa = c.cav_src * (dua * c.idx + dva * c.idx);
    const double fb = c.cav_src * (dub * c.idx + dvb * c.idx);
    const bool out_a = gi >= 1, out_b = gi + 1 <= nx;
    if (out_a && out_b) {
      *reinterpret_cast<double2*>(f + o) = make_double2(fa, fb);
    } else {
      if (out_a) f[o] = fa;
      if (out_b) f[o + 1] = fb;
    }
    m = fmax(out_a ? fabs(fa) : 0.0, out_b ? fabs(fb) : 0.0);
  }
  block_max_to_shard<256>(m, srcmax, (blockIdx.y * gridDim.x + blockIdx.x) % RES_SHARDS);
}

// Sum of per-block partials in a fixed order (one block).
__global__ __launch_bounds__(256) void sum_partials_kernel(const double* __restrict__ partials, int n,
                                                           double* __restrict__ out) {
  double s = 0.0;
  for (int k = threadIdx.x; k < n; k += 256) s += partials[k];
  s = block_sum<256>(s);
  if (threadIdx.x == 0) out[0] = s;
}

// channel-01.cpp:621-628 / backwards_step-01.cpp:844-865: subtract the mean
// over fluid cells, and reduce max|f| (channel-01.cpp:643-646,
// backwards_step-01.cpp:880-887) into the srcmax shards in the same pass.
__global__ __launch_bounds__(256) void subtract_mean_kernel(Geo g, Coef c, double* __restrict__ f,
                                                            const double* __restrict__ total, double count,
                                                            double* __restrict__ srcmax) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j = g.j0 + blockIdx.y * 4 + (threadIdx.x >> 6);
  const int nx = g.nx, ny = g.ny;
  double m = 0.0;
  if (i >= 1 && i <= nx && j >= 1 && j <= ny && j <= g.j1 && is_fluid(c, nx, ny, j, i)) {
    const double mean = total[0] / count;
    const double v = f[at(g, j, i)] - mean;
    f[at(g, j, i)] = v;
    m = fabs(v);
  }
  block_max_to_shard<256>(m, srcmax, (blockIdx.y * gridDim.x + blockIdx.x) % RES_SHARDS);
}

// max|f| over the fluid cells the solve iterates on: cavity-01.cpp:628,
// channel-01.cpp:643-646, backwards_step-01.cpp:880-887 (when the source was
// set from the host rather than built by source_kernel / subtract_mean_kernel).
__global__ __launch_bounds__(256) void srcmax_kernel(Geo g, Coef c, const double* __restrict__ f,
                                                     double* __restrict__ srcmax) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j = g.j0 + blockIdx.y * 4 + (threadIdx.x >> 6);
  const int nx = g.nx, ny = g.ny;
  double m = 0.0;
  if (i >= 1 && i <= nx && j >= 1 && j <= ny && j <= g.j1 && is_fluid(c, nx, ny, j, i)) m = fabs(f[at(g, j, i)]);
  block_max_to_shard<256>(m, srcmax, (blockIdx.y * gridDim.x + blockIdx.x) % RES_SHARDS);
}

// Tolerance of the solve from max|f| (cavity-01.cpp:632, channel-01.cpp:647,
// backwards_step-01.cpp:888) and the value the loop is primed with
// (cavity-01.cpp:618: 1.0; channel-01.cpp:649: tol + 1).
__global__ void tol_kernel(Coef c, const double* __restrict__ srcmax, double* __restrict__ tol) {
  if (threadIdx.x != 0) return;
  double m = 0.0;
  for (int k = 0; k < RES_SHARDS; ++k) m = fmax(m, srcmax[k * SHARD_STRIDE]);
  tol[2] = m;  // max|f| over the interior: the proof-mode test's F
  if (c.case_id == CAVITY) {
    tol[0] = c.tol_factor * m;
    tol[1] = 1.0;
  } else {
    double t = c.tol_factor * (m > 0 ? m : 1.0);
    if (t < c.abs_tol) t = c.abs_tol;
    tol[0] = t;
    tol[1] = t + 1.0;
  }
}


}  // namespace cfd

#include "march.hpp"

namespace cfd {

// Sequential sums in the reference's loop order: seqsum.hip (seq_sum_launch).

// ------------------------------------------- Poisson, exact lexicographic --
//
// The reference's own SOR ordering (Gauss-Seidel sweep in j-then-i order,
// ghosts/solids refreshed after each sweep, residual after the refresh —
// cavity-01.cpp:635-678, channel-01.cpp:652-682, backwards_step-01.cpp:893-931),
// reproduced bit for bit on the GPU as a pipelined wavefront:
//   * cell (j,i) at iteration k is computed at step tau = i + j + 3k; its W/S
//     inputs (iteration k) were computed at tau-1, its E/N/self inputs
//     (iteration k-1) at tau-2 / tau-3; iteration k is stored in X[k & 1];
//   * ghost / solid neighbours are evaluated from stored iteration-(k-1)
//     values with the reference's refresh rules (all their inputs lie within
//     distance 2, computed by tau-1);
//   * in the same step each cell also evaluates the residual of its own
//     iteration k-1 (all inputs complete by tau-1 and not yet overwritten);
//   * iteration k's max-norm residual is complete once the last diagonal has
//     passed; the first k with residual <= tol ends the solve — cells near the
//     origin have run ahead by then, so the solve restores its initial field
//     and replays exactly k iterations (no convergence test on the replay).
// One persistent workgroup runs the whole solve (reference-sized grids).

constexpr int LEX_WIN = 4096;  // residual window (iterations in flight)

template <int CASE>
__device__ __forceinline__ double lex_value(const Coef& c, int nx, int ny, const Geo& g, const double* X, int j, int i,
                                            double self_old, bool from_self) {
  // value of cell (j,i) at the iteration stored in X, as the SOR sweep sees it:
  // interior fluid -> stored; ghost -> refresh rule; solid -> average of fluid
  // neighbours (backwards_step-01.cpp:708-738); cavity ghosts are stored zeros.
  if (CASE == CAVITY) return X[at(g, j, i)];
  const bool jin = j >= 1 && j <= ny, iin = i >= 1 && i <= nx;
  if (jin && iin) {
    if (CASE != BACKSTEP || is_fluid(c, nx, ny, j, i)) return X[at(g, j, i)];
    double sum = 0.0;
    int n = 0;
    if (i > 1 && is_fluid(c, nx, ny, j, i - 1)) { sum += X[at(g, j, i - 1)]; n++; }
    if (i < nx && is_fluid(c, nx, ny, j, i + 1)) { sum += X[at(g, j, i + 1)]; n++; }
    if (j > 1 && is_fluid(c, nx, ny, j - 1, i)) { sum += X[at(g, j - 1, i)]; n++; }
    if (j < ny && is_fluid(c, nx, ny, j + 1, i)) { sum += X[at(g, j + 1, i)]; n++; }
    return n > 0 ? sum / n : X[at(g, j, i)];
  }
  // ghost adjacent to a fluid cell: mirrors that cell (or 0 at the outlet)
  if (i == nx + 1 && jin) return 0.0;
  (void)from_self;
  return self_old;
}

template <int CASE>
__global__ __launch_bounds__(1024) void poisson_lex_kernel(Geo g, Coef c, double* __restrict__ X0,
                                                           double* __restrict__ X1, const double* __restrict__ p0,
                                                           const double* __restrict__ f, const double* __restrict__ tolv,
                                                           int max_iters, int* __restrict__ out_iters,
                                                           double* __restrict__ out_res) {
  __shared__ double win[LEX_WIN];
  __shared__ int s_stop, s_kmax, s_replay;
  const int t = threadIdx.x, NT = blockDim.x;
  const int nx = g.nx, ny = g.ny;
  const double tol = tolv[0];
  const int ncell = nx * ny;
  const int dmax = nx + ny;  // largest i + j
  for (int q = t; q < LEX_WIN; q += NT) win[q] = 0.0;
  if (t == 0) {
    s_stop = 0;
    s_replay = 0;
    s_kmax = max_iters;
  }
  __syncthreads();
  if (!(tolv[1] > tol) || max_iters == 0) {  // loop never entered (cavity-01.cpp:635)
    if (t == 0) { *out_iters = 0; *out_res = tolv[1]; }
    return;
  }
  int tau = 0;
  for (;;) {
    const int kmax = s_kmax;
    const bool replay = s_replay != 0;
    // one wavefront step
    for (int e = t; e < ncell; e += NT) {
      const int jj = e / nx, j = jj + 1, i = e - jj * nx + 1;
      const int r = tau - i - j;
      if (r < 3 || r % 3 != 0) continue;
      const int k = r / 3;  // this step: residual of k-1, update to k
      if (k - 1 > kmax) continue;
      if (!is_fluid(c, nx, ny, j, i)) continue;
      const double* Xo = ((k - 1) & 1) ? X1 : X0;  // iteration k-1
      double* Xn = (k & 1) ? X1 : X0;              // iteration k
      const double self = Xo[at(g, j, i)];
      const double fc = f[at(g, j, i)];
      const double oE = lex_value<CASE>(c, nx, ny, g, Xo, j, i + 1, self, true);
      const double oN = lex_value<CASE>(c, nx, ny, g, Xo, j + 1, i, self, true);
      const double oW = lex_value<CASE>(c, nx, ny, g, Xo, j, i - 1, self, true);
      const double oS = lex_value<CASE>(c, nx, ny, g, Xo, j - 1, i, self, true);
      if (k >= 2 && !replay) {
        const double rv = fabs(residual_at<CASE>(c, nx, ny, j, i, self, oW, oE, oS, oN, fc));
        atomicMax(reinterpret_cast<unsigned long long*>(&win[(k - 1) % LEX_WIN]),
                  (unsigned long long)__double_as_longlong(rv));
      }
      if (k <= kmax) {
        // W/S: iteration k if interior fluid (already swept), else the refreshed value of k-1
        const bool wf = is_fluid(c, nx, ny, j, i - 1), sf = is_fluid(c, nx, ny, j - 1, i);
        const double pW = wf ? Xn[at(g, j, i - 1)] : oW;
        const double pS = sf ? Xn[at(g, j - 1, i)] : oS;
        Xn[at(g, j, i)] = sor_update<CASE>(c, nx, ny, j, i, self, pW, oE, pS, oN, fc);
      }
    }
    __syncthreads();
    // iteration kc's residual is complete after the step with tau = dmax + 3(kc+1)
    if (t == 0) {
      const int r = tau - dmax;
      if (r >= 6 && r % 3 == 0) {
        const int kc = r / 3 - 1;
        if (replay) {
          if (kc >= kmax) s_stop = 1;
        } else {
          const double rk = win[kc % LEX_WIN];
          win[kc % LEX_WIN] = 0.0;  // slot reused by iteration kc + LEX_WIN
          if (!(rk > tol) || kc >= max_iters) {
            *out_iters = kc;
            *out_res = rk;
            if (kc < max_iters && tau - 3 * kc > 3) {
              // converged at kc while later iterations already ran: replay exactly kc
              s_replay = 1;
              s_kmax = kc;
            } else {
              s_stop = 1;
            }
          }
        }
      }
    }
    __syncthreads();
    if (s_stop) break;
    if (s_replay && !replay) {  // restore the solve's initial field and restart the wavefront
      for (int e = t; e < (int)((size_t)g.nrows * g.pitch); e += NT) X0[e] = p0[e];
      __syncthreads();
      tau = 0;
      continue;
    }
    ++tau;
  }
  // refresh ghosts / solids of the final field from its interior (reference order:
  // walls read pre-refresh solids, so compute everything first, then write)
  if (CASE != CAVITY) {
    const int K = *out_iters;
    double* Xf = (K & 1) ? X1 : X0;
    const double* Xp = (K & 1) ? X0 : X1;  // iteration K-1
    const int W2 = nx + 2, n2 = (ny + 2) * (nx + 2);
    __syncthreads();
    if (CASE == BACKSTEP && K >= 2) {
      // solid cells as the sweep of iteration K left them: refreshed from iteration K-1
      for (int e = t; e < n2; e += NT) {
        const int j = e / W2, i = e - j * W2;
        if (j >= 1 && j <= ny && i >= 1 && i <= nx && !is_fluid(c, nx, ny, j, i))
          Xf[at(g, j, i)] = lex_value<CASE>(c, nx, ny, g, Xp, j, i, 0.0, false);
      }
      __syncthreads();
    }
    for (int pass = 0; pass < 2; ++pass) {
      for (int e = t; e < n2; e += NT) {
        const int j = e / W2, i = e - j * W2;
        const bool jin = j >= 1 && j <= ny, iin = i >= 1 && i <= nx;
        double v;
        bool set = true;
        if (i == 0 && jin) v = Xf[at(g, j, 1)];
        else if (i == nx + 1 && jin) v = 0.0;
        else if (j == 0 && iin) v = Xf[at(g, 1, i)];
        else if (j == ny + 1 && iin) v = Xf[at(g, ny, i)];
        else set = false;
        if (pass == 0 && set) Xf[at(g, j, i)] = v;  // walls first: they read interior cells
        if (pass == 1 && CASE == BACKSTEP && jin && iin && !is_fluid(c, nx, ny, j, i)) {
          double sum = 0.0;
          int n = 0;
          if (i > 1 && is_fluid(c, nx, ny, j, i - 1)) { sum += Xf[at(g, j, i - 1)]; n++; }
          if (i < nx && is_fluid(c, nx, ny, j, i + 1)) { sum += Xf[at(g, j, i + 1)]; n++; }
          if (j > 1 && is_fluid(c, nx, ny, j - 1, i)) { sum += Xf[at(g, j - 1, i)]; n++; }
          if (j < ny && is_fluid(c, nx, ny, j + 1, i)) { sum += Xf[at(g, j + 1, i)]; n++; }
          if (n > 0) Xf[at(g, j, i)] = sum / n;
        }
      }
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------ corrector --

// cavity-01.cpp:695-711 / channel-01.cpp:693-702 / backwards_step-01.cpp:944-976.
__global__ __launch_bounds__(256) void correct_kernel(Geo g, Coef c, const double* __restrict__ p,
                                                      const double* __restrict__ us, const double* __restrict__ vs,
                                                      double* __restrict__ u, double* __restrict__ v) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j = g.j0 + blockIdx.y * 4 + (threadIdx.x >> 6);
  const int nx = g.nx, ny = g.ny;
  if (j > g.j1 || j < 1 || j > ny) return;
  const bool step = c.case_id == BACKSTEP, cav = c.case_id == CAVITY;
  const size_t o = at(g, j, i);
  const size_t P = (size_t)g.pitch;
  if (i >= 1 && i <= nx - 1) {
    const double dp = p[o + 1] - p[o];
    const double a = us[o] - c.cav_corr * dp;
    const double b = us[o] - c.open_cu * dp;
    const bool valid = !step || (i == nx - 1) || is_fluid(c, nx, ny, j, i) || is_fluid(c, nx, ny, j, i + 1);
    u[o] = cav ? a : (valid ? b : 0.0);
  }
  if (i >= 1 && i <= nx && j <= ny - 1) {
    const double dp = p[o + P] - p[o];
    const double a = vs[o] - c.cav_corr * dp;
    const double b = vs[o] - c.open_cv * dp;
    const bool valid = !step || (j == ny - 1) || is_fluid(c, nx, ny, j, i) || is_fluid(c, nx, ny, j + 1, i);
    v[o] = cav ? a : (valid ? b : 0.0);
  }
}

// ------------------------------------------------------ post-processing --

// cavity-01.cpp:717-733 / backwards_step-01.cpp:981-1009 (cell-centre
// velocities) fused with cavity-01.cpp:750-764 / channel-01.cpp:743-757
// (kinetic-energy partial sums and max |div|).
__global__ __launch_bounds__(256) void centers_stats_kernel(Geo g, Coef c, const double* __restrict__ u,
                                                            const double* __restrict__ v, double* __restrict__ uc,
                                                            double* __restrict__ vc, double* __restrict__ ke_part,
                                                            double* __restrict__ divmax) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j = g.j0 + blockIdx.y * 4 + (threadIdx.x >> 6);
  const int nx = g.nx, ny = g.ny;
  double ke = 0.0, dv = 0.0;
  if (i >= 1 && i <= nx && j >= 1 && j <= ny && j <= g.j1) {
    const bool fl = is_fluid(c, nx, ny, j, i);
    const size_t o = at(g, j, i);
    const size_t P = (size_t)g.pitch;
    const double uo = u[o], uw = u[o - 1], vo = v[o], vs_ = v[o - P];
    const double a = 0.5 * (uw + uo);
    const double b = 0.5 * (vs_ + vo);
    const double dc = (uo - uw + vo - vs_) * c.idx;
    const double dop = (uo - uw) * c.idx + (vo - vs_) * c.idy;
    ke = fl ? 0.5 * (a * a + b * b) : 0.0;
    dv = fl ? fabs(c.case_id == CAVITY ? dc : dop) : 0.0;
    uc[o] = fl ? a : 0.0;
    vc[o] = fl ? b : 0.0;
  }
  const int blin = blockIdx.y * gridDim.x + blockIdx.x;
  const double s = block_sum<256>(ke);
  if (threadIdx.x == 0) ke_part[blin] = s;
  __syncthreads();
  block_max_to_shard<256>(dv, divmax, blin % RES_SHARDS);
}

}  // namespace cfd
