// seqsum.hpp — launcher of the reference-order sequential sums (seqsum.hip).
#pragma once

#include "device.hpp"

namespace cfd {

// Sum over the strip's interior cells in the reference's loop order (j outer,
// i inner; the step's solid cells skipped) with one rounding per term, as the
// reference's loop: mode 0 = a (the source, channel-01.cpp:620-628,
// backwards_step-01.cpp:843-866), mode 1 = 0.5 (a^2 + b^2) (the kinetic
// energy, cavity-01.cpp:750-755). accumulate: continue from out[0] (strips in
// order), else start from 0. ws: seq_sum_workspace(terms) bytes of device
// memory (the chunk records); serial_count (device, may be null): += the
// chunks that ran as the plain chain. Returns the number of chunks.
long long seq_sum_launch(const Geo& g, const Coef& c, const double* a, const double* b, int mode, double* out,
                         int accumulate, void* ws, size_t ws_bytes, int* serial_count, hipStream_t st);
size_t seq_sum_workspace(long long n_terms);

}  // namespace cfd
