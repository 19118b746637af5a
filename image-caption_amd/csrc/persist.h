// capgen — persistent multi-GEMM launches (experiments; persist.hip).
#pragma once
#include "gemm.h"

namespace capgen {

// H = relu(X . W1^T + b1) (g1: M x fe x d, C = H) and Y = H . W2^T (g2: M x d x fe, A = H) in one
// persistent launch of `grid` workgroups (64x64 tiles, row-block dependency counters).
// acquire = 0 drops the consumer's agent acquire (diagnostic only).
void ffn_persistent(const GemmArgs& g1, const GemmArgs& g2, int grid, int acquire, hipStream_t s);
// spins that gave up since the last reset (0 in a correct run)
int ffn_persistent_giveups(bool reset);

}  // namespace capgen
