// Reconstruction of the round-1 source_kernel form that faulted on the first
// GPU run (DESIGN.md "GPU memory fault, round 1"): the reference's branch
// structure (cavity-01.cpp:622-630, channel-01.cpp:613-619,
// backwards_step-01.cpp:830-841) as an if / else-if / else chain with one
// store per branch. COMPILE-ONLY: it is never launched here (a faulting
// kernel can reset the GPU host); `make` writes the gfx950 ISA next to it and
// isa_stores.py lists each global_store with the block it sits in and the
// exec mask that block runs under. The shipped kernel (csrc/kernels.hpp
// source_kernel) forms the address once and selects the value instead.
#include "../../computational-fluid-dynamics_amd/csrc/kernels.hpp"

namespace cfd {
__global__ __launch_bounds__(256) void source_kernel_ifelse(Geo g, Coef c, const double* __restrict__ us,
                                                            const double* __restrict__ vs, double* __restrict__ f,
                                                            double* __restrict__ partials) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j = g.j0 + blockIdx.y * 4 + (threadIdx.x >> 6);
  const int nx = g.nx, ny = g.ny;
  double val = 0.0;
  if (i >= 1 && i <= nx && j >= 1 && j <= ny && j <= g.j1) {
    const size_t o = at(g, j, i);
    const double du = us[o] - us[o - 1];
    const double dv = vs[o] - vs[o - (size_t)g.pitch];
    if (c.case_id == CAVITY) {
      val = c.cav_src * (du * c.idx + dv * c.idx);
      f[o] = val;
    } else if (is_fluid(c, nx, ny, j, i)) {
      val = c.open_src * (du * c.idx + dv * c.idy);
      f[o] = val;
    } else {
      f[o] = 0.0;
    }
  }
  if (c.case_id != CAVITY) {
    const double s = block_sum<256>(val);
    if (threadIdx.x == 0) partials[blockIdx.y * gridDim.x + blockIdx.x] = s;
  }
}
}  // namespace cfd
