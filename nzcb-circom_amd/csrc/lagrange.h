// Lagrange-basis SRS of a PLONK domain from the zkey's PTau (csrc/lagrange.hip).
#pragma once
#include "ec.h"

namespace nzcb {

// out[0..n) = [L_k(tau)] for the 2^logn-th roots of unity, out[n] = [tau^n] - [1],
// out[n+1] = [tau^(n+1)] - [tau] (affine, PTau's LEM layout). ptau: ptau_n >= n + 2 points
// in HBM. Synchronous on `st`.
void lagrange_basis(const G1Affine* ptau, size_t ptau_n, int logn, G1Affine* out, hipStream_t st);

}  // namespace nzcb
