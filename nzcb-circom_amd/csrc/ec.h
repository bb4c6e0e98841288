// BN254 G1 (y^2 = x^3 + 3) point arithmetic for the MSM kernels.
//
// Replaces wasmcurves' g1m_* Jacobian add/double/mixed-add (SURVEY.md §8a
// row a13). Buckets use extended-Jacobian "XYZZ" coordinates
// (x = X/ZZ, y = Y/ZZZ): a mixed add into a bucket costs 8M+2S with no
// inversion, and every special case (empty bucket, P == Q, P == -Q) is a cheap
// branch on ZZ / the two differences, so adding the same base twice or a point
// and its negation inside one bucket is exact.
// Affine points are the zkey's 64-byte LEM layout (x || y, Montgomery, LE);
// (0,0) encodes infinity (not on the curve, since 0 != 0^3 + 3).
#pragma once
#include "field.h"

namespace nzcb {

struct G1Affine {
  Fq x, y;
  NZ_HD bool is_inf() const { return x.is_zero() && y.is_zero(); }
};

struct G1xyzz {
  Fq X, Y, ZZ, ZZZ;
  NZ_HD static G1xyzz inf() {
    G1xyzz r;
    r.X = Fq::one();
    r.Y = Fq::one();
    r.ZZ = Fq::zero();
    r.ZZZ = Fq::zero();
    return r;
  }
  NZ_HD bool is_inf() const { return ZZ.is_zero(); }
};

NZ_HD G1xyzz xyzz_from_affine(const G1Affine& p) {
  if (p.is_inf()) return G1xyzz::inf();
  G1xyzz r;
  r.X = p.x;
  r.Y = p.y;
  r.ZZ = Fq::one();
  r.ZZZ = Fq::one();
  return r;
}

// dbl-2008-s-1 (a = 0)
NZ_HD G1xyzz xyzz_dbl(const G1xyzz& p) {
  if (p.is_inf() || p.Y.is_zero()) return G1xyzz::inf();
  Fq U = dbl(p.Y);
  Fq V = sqr(U);
  Fq W = U * V;
  Fq S = p.X * V;
  Fq X2 = sqr(p.X);
  Fq M = X2 + dbl(X2);
  G1xyzz r;
  r.X = sqr(M) - dbl(S);
  r.Y = M * (S - r.X) - W * p.Y;
  r.ZZ = V * p.ZZ;
  r.ZZZ = W * p.ZZZ;
  return r;
}

// mdbl-2008-s-1: double an affine point into XYZZ
NZ_HD G1xyzz xyzz_mdbl(const Fq& x, const Fq& y) {
  if (y.is_zero()) return G1xyzz::inf();
  Fq U = dbl(y);
  Fq V = sqr(U);
  Fq W = U * V;
  Fq S = x * V;
  Fq X2 = sqr(x);
  Fq M = X2 + dbl(X2);
  G1xyzz r;
  r.X = sqr(M) - dbl(S);
  r.Y = M * (S - r.X) - W * y;
  r.ZZ = V;
  r.ZZZ = W;
  return r;
}

// Rare special cases (P == Q inside an addition). Out-of-line calls shrink the code
// but cost registers (ABI) and occupancy: measured on MI355X the accumulate kernel went
// from 3.6 to 6.6 ms with them out of line, so they stay inline unless NZ_RARE_NOINLINE.
#if defined(__HIP_DEVICE_COMPILE__) && defined(NZ_RARE_NOINLINE)
static __device__ __noinline__ void xyzz_mdbl_rare(const Fq& x, const Fq& y, G1xyzz* out) {
  *out = xyzz_mdbl(x, y);
}
static __device__ __noinline__ void xyzz_dbl_rare(const G1xyzz& p, G1xyzz* out) { *out = xyzz_dbl(p); }
#define NZ_MDBL_RARE(x, y) ([&] { G1xyzz r_; xyzz_mdbl_rare((x), (y), &r_); return r_; }())
#define NZ_DBL_RARE(p) ([&] { G1xyzz r_; xyzz_dbl_rare((p), &r_); return r_; }())
#else
#define NZ_MDBL_RARE(x, y) xyzz_mdbl((x), (y))
#define NZ_DBL_RARE(p) xyzz_dbl((p))
#endif

// madd-2008-s: p (XYZZ) + q (affine, not infinity)
NZ_HD G1xyzz xyzz_add_affine(const G1xyzz& p, const Fq& qx, const Fq& qy) {
  if (p.is_inf()) {
    G1xyzz r;
    r.X = qx;
    r.Y = qy;
    r.ZZ = Fq::one();
    r.ZZZ = Fq::one();
    return r;
  }
  Fq U2 = qx * p.ZZ;
  Fq S2 = qy * p.ZZZ;
  Fq P = U2 - p.X;
  Fq R = S2 - p.Y;
  if (P.is_zero()) {
    if (R.is_zero()) return NZ_MDBL_RARE(qx, qy);
    return G1xyzz::inf();
  }
  Fq PP = sqr(P);
  Fq PPP = P * PP;
  Fq Q = p.X * PP;
  G1xyzz r;
  r.X = sqr(R) - PPP - dbl(Q);
  r.Y = R * (Q - r.X) - p.Y * PPP;
  r.ZZ = p.ZZ * PP;
  r.ZZZ = p.ZZZ * PPP;
  return r;
}

// add-2008-s: XYZZ + XYZZ
NZ_HD G1xyzz xyzz_add(const G1xyzz& p, const G1xyzz& q) {
  if (p.is_inf()) return q;
  if (q.is_inf()) return p;
  Fq U1 = p.X * q.ZZ;
  Fq U2 = q.X * p.ZZ;
  Fq S1 = p.Y * q.ZZZ;
  Fq S2 = q.Y * p.ZZZ;
  Fq P = U2 - U1;
  Fq R = S2 - S1;
  if (P.is_zero()) {
    if (R.is_zero()) return NZ_DBL_RARE(p);
    return G1xyzz::inf();
  }
  Fq PP = sqr(P);
  Fq PPP = P * PP;
  Fq Q = U1 * PP;
  G1xyzz r;
  r.X = sqr(R) - PPP - dbl(Q);
  r.Y = R * (Q - r.X) - S1 * PPP;
  r.ZZ = p.ZZ * q.ZZ * PP;
  r.ZZZ = p.ZZZ * q.ZZZ * PPP;
  return r;
}

NZ_HD G1xyzz xyzz_neg(const G1xyzz& p) {
  G1xyzz r = p;
  r.Y = neg(p.Y);
  return r;
}

// k * p for a small non-negative integer k (double-and-add, MSB first)
NZ_HD G1xyzz xyzz_mul_small(const G1xyzz& p, uint32_t k) {
  G1xyzz r = G1xyzz::inf();
  for (int b = 31; b >= 0; b--) {
    r = xyzz_dbl(r);
    if ((k >> b) & 1u) r = xyzz_add(r, p);
  }
  return r;
}

}  // namespace nzcb
