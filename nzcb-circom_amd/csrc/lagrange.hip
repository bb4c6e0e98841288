// Lagrange-basis SRS from the zkey's PTau, for committing A, B and C from their
// evaluations.
//
// snarkjs commits a polynomial from its coefficients: [p(tau)] = sum_i c_i [tau^i]
// (expTau over the zkey's PTau). For A, B and C the same point is
//   [p(tau)] = sum_k p(w^k) [L_k(tau)] + b_lo ([tau^n] - [1]) + b_hi ([tau^(n+1)] - [tau])
// where p(w^k) are the gate values buildABC gathers and b_lo + b_hi X the blinding factor
// of to4T (k_blind). The commitment, and so the proof, is bit-identical, but the scalars
// are now the witness values, and for nzcp_live most of them are bits, bytes or small
// sums: 0.7 / 1.5 / 0.8 nonzero 17-bit windows per A / B / C value against 15 for the
// random-looking coefficients. The MSM's bucketing drops zero digits, so
// the three commitments cost a tenth of a coefficient-form MSM.
//
// [L_k(tau)] = (1/n) sum_i w^(-ik) [tau^i] is the inverse DFT of the PTau points, computed
// once per context by an elliptic-curve NTT: radix-2 DIT over XYZZ points, where a
// butterfly's twiddle product is a 254-bit double-and-add scalar multiplication. Lanes of
// a wave share their twiddle while a stage has >= 64 groups (its bits are then uniform);
// the last 6 stages use a twiddle per lane.
#include "common.h"
#include "ec.h"
#include "lagrange.h"
#include "ntt.h"

namespace nzcb {
namespace {

constexpr int kLT = 256;

__device__ __forceinline__ uint32_t bitrev(uint32_t x, int bits) { return __brev(x) >> (32 - bits); }

// k * p for a normal-form 254-bit scalar (double-and-add, MSB first)
__device__ G1xyzz xyzz_mul(const G1xyzz& p, const Fr& k) {
  G1xyzz r = G1xyzz::inf();
  for (int b = 253; b >= 0; b--) {
    r = xyzz_dbl(r);
    if ((k.v[b >> 5] >> (b & 31)) & 1u) r = xyzz_add(r, p);
  }
  return r;
}

// tw[k] = w^-k (normal form) for k < half
__global__ void k_lag_twiddles(Fr* __restrict__ tw, Fr winv, size_t half) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= half) return;
  tw[k] = from_mont(pow_u64(winv, (uint64_t)k));
}

// X[bitrev(i)] = (1/n) PTau[i]
__global__ void k_lag_load(const G1Affine* __restrict__ ptau, size_t n, int logn, Fr inv_n, G1xyzz* __restrict__ X) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  X[bitrev((uint32_t)i, logn)] = xyzz_mul(xyzz_from_affine(ptau[i]), inv_n);
}

// stage s: blocks of 2 half = 2^(s+1) points; butterfly (u, v) -> (u + w v, u - w v)
__global__ void __launch_bounds__(kLT) k_lag_stage(G1xyzz* __restrict__ X, size_t n, int logn, int s,
                                                   const Fr* __restrict__ tw) {
  const size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n / 2) return;
  const size_t half = (size_t)1 << s;
  const size_t groups = n / (2 * half);
  size_t g, j;
  if (groups >= 64) {  // consecutive threads: same j (a wave-uniform twiddle), different groups
    j = b / groups;
    g = b % groups;
  } else {
    g = b / half;
    j = b % half;
  }
  const size_t i0 = g * 2 * half + j, i1 = i0 + half;
  const G1xyzz u = X[i0];
  G1xyzz v = X[i1];
  if (j) v = xyzz_mul(v, tw[j << (logn - 1 - s)]);
  X[i0] = xyzz_add(u, v);
  X[i1] = xyzz_add(u, xyzz_neg(v));
}

__device__ G1Affine to_affine_dev(const G1xyzz& p) {
  G1Affine r;
  if (p.is_inf()) {
    r.x = Fq::zero();
    r.y = Fq::zero();
    return r;
  }
  r.x = p.X * inverse(p.ZZ);
  r.y = p.Y * inverse(p.ZZZ);
  return r;
}

// out[k] = affine X[k] (k < n); out[n] = [tau^n] - [1], out[n+1] = [tau^(n+1)] - [tau]
__global__ void k_lag_store(const G1xyzz* __restrict__ X, const G1Affine* __restrict__ ptau, size_t n,
                            G1Affine* __restrict__ out) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) {
    out[k] = to_affine_dev(X[k]);
  } else if (k < n + 2) {
    const size_t e = k - n;  // 0: tau^n - 1, 1: tau^(n+1) - tau
    const G1xyzz hi = xyzz_from_affine(ptau[n + e]);
    const G1xyzz lo = xyzz_from_affine(ptau[e]);
    out[k] = to_affine_dev(xyzz_add(hi, xyzz_neg(lo)));
  }
}

}  // namespace

void lagrange_basis(const G1Affine* ptau, size_t ptau_n, int logn, G1Affine* out, hipStream_t st) {
  const size_t n = size_t(1) << logn;
  if (logn < 1 || logn > 26) throw Error(NZCB_ERR_ARG, "lagrange basis: bad domain size");
  if (ptau_n < n + 2) throw Error(NZCB_ERR_ARG, "lagrange basis: PTau holds fewer than n + 2 points");
  DevBuf<G1xyzz> X(n);
  DevBuf<Fr> tw(n / 2);
  const Fr w = fr_root_of_unity(logn);
  Fr nn = Fr::zero();
  nn.v[0] = (uint32_t)n;
  const Fr inv_n = from_mont(inverse(to_mont(nn)));
  hipLaunchKernelGGL(k_lag_twiddles, dim3(grid_for(n / 2, kLT)), dim3(kLT), 0, st, tw.p, inverse(w), n / 2);
  hipLaunchKernelGGL(k_lag_load, dim3(grid_for(n, kLT)), dim3(kLT), 0, st, ptau, n, logn, inv_n, X.p);
  NZ_HIP(hipGetLastError());
  for (int s = 0; s < logn; s++) {
    hipLaunchKernelGGL(k_lag_stage, dim3(grid_for(n / 2, kLT)), dim3(kLT), 0, st, X.p, n, logn, s, tw.p);
    NZ_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(k_lag_store, dim3(grid_for(n + 2, kLT)), dim3(kLT), 0, st, X.p, ptau, n, out);
  NZ_HIP(hipGetLastError());
  NZ_HIP(hipStreamSynchronize(st));  // X and tw are freed on return
}

}  // namespace nzcb
