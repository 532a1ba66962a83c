// open.hpp — launcher of the open cases' proof-mode SOR launches (open.hip).
#pragma once

#include "march.hpp"

namespace cfd {

// One launch of `ns` (3 or 4) red-black iterations k .. k+ns-1 of the channel /
// backwards step with the proof-mode convergence test, tiled by `pl` like
// poisson_multi_kernel; testing [ka, kb] first (flags as poisson_multi_kernel).
void open_proof_launch(int case_id, int ns, const Geo& g, const Coef& c, const double* pin, double* pout,
                       const double* f, const PoissonCtl& ctl, int k, int ka, int kb, const PairPlan& pl, int flags,
                       hipStream_t st);

}  // namespace cfd
