// smlex.hpp — launcher of the reference-order SOR solve of a reference-sized
// grid in one workgroup (smlex.hip).
#pragma once

#include "device.hpp"

namespace cfd {

constexpr int SMLEX_THREADS = 1024;
constexpr int SMLEX_CELLS = 20160;  // (nx+2)(ny+2) at most: p in LDS (157.5 KiB)
constexpr int SMLEX_MAXC = 5;       // cells of one colour per thread, at most (their state in registers)
constexpr int SMLEX_NF = 512;       // per-iteration exceedance flags in flight (ring)
constexpr int SMLEX_NCK = 4;        // checkpoint buffers (global memory, SMLEX_NCK x (nx+2)(ny+2) doubles)

// Grids the kernel takes: p fits the LDS, each thread's cells their registers, the iterations in flight fit
// the flag ring, and the step's block has a corner cell with two fluid
// neighbours (the same geometries as the multi-block reference-order march).
bool smlex_fits(const Geo& g, const Coef& c);

// Doubles of checkpoint scratch (ck of smlex_launch) a grid needs.
size_t smlex_ck_doubles(int nx, int ny);

// Checkpoint spacing (iterations) for a grid: three intervals cover the
// iterations the first cell runs ahead of the last one.
int smlex_interval(int nx, int ny);

// The whole solve (cavity-01.cpp:633-678, channel-01.cpp:652-682,
// backwards_step-01.cpp:893-931) on p in place: iteration count and the final
// field's max-norm residual to out_iters / out_res. ck: checkpoint scratch.
void smlex_launch(int case_id, const Geo& g, const Coef& c, double* p, const double* f, const double* tolv,
                  int max_iters, double* ck, int* out_iters, double* out_res, hipStream_t st);

}  // namespace cfd
