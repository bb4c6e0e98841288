// BN254 Fq in a redundant radix 2^29 (9 limbs, Montgomery R = 2^261) for the MSM
// bucket accumulation.
//
// Why: on gfx950 v_mad_u64_u32 and v_addc_co_u32 both issue at 4 cycles per wave64
// instruction (profiles/r1_isa_bench.txt). With 32-bit limbs every partial product
// needs mad + addc. With 29-bit limbs a partial product is < 2^58 (< 2^60 with one
// bit of limb slack), so a whole column (<= 18 products plus the carry) stays below
// 2^64 in one accumulator. That is one v_mad_u64_u32 per partial product, no carry
// instruction and no final subtraction. tools/mul29bench.hip measures 133.6 G
// products/s against 103.2 for csrc/field.h.
//
// Value invariants (x < 2^257 for every product input, 10p = 0.945 * 2^257):
//   mul29(a, b): a, b < 2^257 with limbs < 2^30  ->  result < 2p, limbs < 2^29
//   sub29<K>(a, b) = a + K - b with K = k*p in "borrowed" limbs (every limb >= 2^29 - 1,
//   so no limb goes negative), b < K, a and b normalized; result normalized
// Only add/sub/mul are needed by the XYZZ mixed addition (msm.hip).
#pragma once
#include "field.h"

namespace nzcb {

struct F29 {
  uint32_t v[9];
};

struct Fq29 {
  static constexpr uint32_t MASK = (1u << 29) - 1;
  static constexpr uint32_t INV = 0x04866389u;  // -p^-1 mod 2^29
  static constexpr uint32_t P[9] = {0x187cfd47u, 0x010460b6u, 0x1c72a34fu, 0x02d522d0u, 0x1585d978u,
                                    0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
  // k*p in borrowed form (k = 2, 4, 6, 8)
  static constexpr uint32_t K2[9] = {0x30f9fa8eu, 0x2208c16cu, 0x38e5469du, 0x25aa45a0u, 0x2b0bb2efu,
                                     0x25b68180u, 0x214dc281u, 0x3cb84c67u, 0x0060c89bu};
  static constexpr uint32_t K4[9] = {0x21f3f51cu, 0x241182dau, 0x31ca8d3bu, 0x2b548b42u, 0x361765dfu,
                                     0x2b6d0301u, 0x229b8503u, 0x397098cfu, 0x00c19138u};
  static constexpr uint32_t K6[9] = {0x32edefaau, 0x261a4447u, 0x2aafd3d9u, 0x30fed0e4u, 0x212318cfu,
                                     0x31238483u, 0x23e94785u, 0x3628e537u, 0x012259d5u};
  static constexpr uint32_t K8[9] = {0x23e7ea38u, 0x282305b5u, 0x23951a77u, 0x36a91686u, 0x2c2ecbbfu,
                                     0x36da0604u, 0x25370a07u, 0x32e1319fu, 0x01832272u};
  static constexpr uint32_t ONE[9] = {0x157ccc21u, 0x141c2758u, 0x185230d3u, 0x014c0419u, 0x0aa36fb9u,
                                      0x1d4240ceu, 0x11d54c07u, 0x052ac7a8u, 0x000dc836u};  // 2^261 mod p
  static constexpr uint32_t C256[9] = {0x058f0d9du, 0x1aea1c6eu, 0x11c2cf74u, 0x11d651ebu, 0x1462c0a7u,
                                       0x11b7bc3cu, 0x1cbd99bau, 0x183340fbu, 0x000e0a77u};  // 2^256 mod p
};

// BN254 Fr in the same radix (the NTT's twiddle products, ntt.hip). r = 1 + 2^28 t,
// so -r^-1 mod 2^29 = 2^28 - 1.
struct Fr29 {
  static constexpr uint32_t MASK = (1u << 29) - 1;
  static constexpr uint32_t INV = 0x0fffffffu;
  static constexpr uint32_t P[9] = {0x10000001u, 0x1f0fac9fu, 0x0e5c2450u, 0x07d090f3u, 0x1585d283u,
                                    0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
  // 2r in borrowed form (every limb >= 2^29 - 1), for sub29
  static constexpr uint32_t K2[9] = {0x20000002u, 0x3e1f593eu, 0x3cb848a0u, 0x2fa121e5u, 0x2b0ba505u,
                                     0x25b68180u, 0x214dc281u, 0x3cb84c67u, 0x0060c89bu};
  static constexpr uint32_t ONE[9] = {0x0fffff57u, 0x1ea70ab4u, 0x052c068bu, 0x17504f49u, 0x0aa8075bu,
                                      0x1d4240ceu, 0x11d54c07u, 0x052ac7a8u, 0x000dc836u};  // 2^261 mod r
  static constexpr uint32_t C256[9] = {0x0ffffffbu, 0x04b1a0e2u, 0x18334a6bu, 0x18ed2b3eu, 0x1462e36fu,
                                       0x11b7bc3cu, 0x1cbd99bau, 0x183340fbu, 0x000e0a77u};  // 2^256 mod r
  // 4r in borrowed form: the NTT butterflies' a + 4r - b for Shoup products b < 3r
  static constexpr uint32_t K4[9] = {0x20000004u, 0x3c3eb27du, 0x39709142u, 0x3f4243ccu, 0x36174a0bu,
                                     0x2b6d0301u, 0x229b8503u, 0x397098cfu, 0x00c19138u};
  // 2^261 - r (mul_shoup: x w - q r = x w + q (2^261 - r) mod 2^261)
  static constexpr uint32_t RP[9] = {0x0fffffffu, 0x00f05360u, 0x11a3dbafu, 0x182f6f0cu, 0x0a7a2d7cu,
                                     0x1d24bf3fu, 0x1f591ebeu, 0x11a3d9cbu, 0x1fcf9bb1u};
  // -r^-1 mod 2^261 (the Shoup quotient of a twiddle from its Montgomery-261 form, ntt.hip)
  static constexpr uint32_t NINV[9] = {0x0fffffffu, 0x170fac9fu, 0x1a446cf0u, 0x0d0c9698u, 0x02391658u,
                                       0x0c144c83u, 0x06cb8e6au, 0x03a1b068u, 0x1273f82fu};
};

// acc + x * y as one v_mad_u64_u32 with acc as its addend. Written as asm so the
// compiler keeps each column one accumulation chain: left to itself it restarts every
// column at 0 and adds the previous column's carry with an extra 64-bit add (about
// 150 v_lshl_add_u64 per XYZZ addition). mad29c takes y from an SGPR (modulus limbs).
#ifndef NZ_MAD_ASM
#define NZ_MAD_ASM 1
#endif
#if defined(__HIP_DEVICE_COMPILE__) && NZ_MAD_ASM
__device__ __forceinline__ void mad29(uint64_t& acc, uint32_t x, uint32_t y) {
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc) : "v"(x), "v"(y) : "vcc");
}
__device__ __forceinline__ void mad29c(uint64_t& acc, uint32_t x, uint32_t y) {
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc) : "v"(x), "s"(y) : "vcc");
}
// two independent mads in one asm statement (mul29x2): the compiler's s_nop between
// inline-asm statements is paid once per pair
__device__ __forceinline__ void mad29x2(uint64_t& acc, uint32_t x, uint32_t y, uint64_t& bcc, uint32_t u,
                                        uint32_t v) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_mad_u64_u32 %1, vcc, %4, %5, %1"
      : "+v"(acc), "+v"(bcc) : "v"(x), "v"(y), "v"(u), "v"(v) : "vcc");
}
__device__ __forceinline__ void mad29cx2(uint64_t& acc, uint32_t x, uint64_t& bcc, uint32_t u, uint32_t y) {
  asm("v_mad_u64_u32 %0, vcc, %2, %4, %0\n\tv_mad_u64_u32 %1, vcc, %3, %4, %1"
      : "+v"(acc), "+v"(bcc) : "v"(x), "v"(u), "s"(y) : "vcc");
}
#else
NZ_HD void mad29(uint64_t& acc, uint32_t x, uint32_t y) { acc += (uint64_t)x * y; }
NZ_HD void mad29c(uint64_t& acc, uint32_t x, uint32_t y) { acc += (uint64_t)x * y; }
NZ_HD void mad29x2(uint64_t& acc, uint32_t x, uint32_t y, uint64_t& bcc, uint32_t u, uint32_t v) {
  acc += (uint64_t)x * y;
  bcc += (uint64_t)u * v;
}
NZ_HD void mad29cx2(uint64_t& acc, uint32_t x, uint64_t& bcc, uint32_t u, uint32_t y) {
  acc += (uint64_t)x * y;
  bcc += (uint64_t)u * y;
}
#endif

NZ_HD F29 f29_const(const uint32_t (&c)[9]);

#ifndef NZ_MAD_COLS
#define NZ_MAD_COLS 1
#endif
#if defined(__HIP_DEVICE_COMPILE__) && NZ_MAD_ASM && NZ_MAD_COLS
#include "f29_cols.h"
#define NZ_F29_COLS 1
#else
#define NZ_F29_COLS 0
#endif


// Shoup's product by a fixed factor (the NTT twiddles): w < r and ws = floor(w 2^261 / r),
// both normalized; x < 2^261 with limbs < 2^30.6. q = floor(x ws / 2^261) from the product
// columns 7..16 only (the dropped columns 0..6 sum to < 2^237, so q is off by at most 1 from
// the exact floor, which is itself floor(x w / r) or one less: x ws / 2^261 > x w / r - 1),
// then x w - q r = x w + q (2^261 - r) mod 2^261 from the low columns 0..8 alone, the exact
// value since it is < 3r < 2^261. Result < 3r, normalized. 143 v_mad_u64_u32 (45 + 53 + 45)
// and no v_mul_lo_u32 against the Montgomery product's 162 + 9 (round 5, the NTT's twiddles).
// A column of the low half is <= 9 (2^59.6 + 2^58) + 2^35 < 2^64, of x ws <= 9 2^59.6 + 2^35.
template <int N>
NZ_HD void mul_shoup_n(const F29 (&x)[N], const F29 (&w)[N], const F29 (&ws)[N], F29 (&out)[N]) {
#if NZ_F29_COLS
  if constexpr (N == 2) {
    mul_shoup2_cols(x[0], w[0], ws[0], x[1], w[1], ws[1], out[0], out[1]);
    return;
  } else if constexpr (N == 1) {
    out[0] = mul_shoup1_cols(x[0], w[0], ws[0]);
    return;
  }
#endif
  using Q = Fr29;
  uint32_t q[N][9];
  uint64_t acc[N];
#pragma unroll
  for (int t = 0; t < N; t++) acc[t] = 0;
#pragma unroll
  for (int c = 7; c < 17; c++) {
#pragma unroll
    for (int j = c > 8 ? c - 8 : 0; j <= (c < 8 ? c : 8); j++) {
      if constexpr (N == 2) {
        mad29x2(acc[0], x[0].v[j], ws[0].v[c - j], acc[1], x[1].v[j], ws[1].v[c - j]);
      } else {
#pragma unroll
        for (int t = 0; t < N; t++) mad29(acc[t], x[t].v[j], ws[t].v[c - j]);
      }
    }
#pragma unroll
    for (int t = 0; t < N; t++) {
      if (c >= 9) q[t][c - 9] = (uint32_t)acc[t] & Q::MASK;
      acc[t] >>= 29;
    }
  }
#pragma unroll
  for (int t = 0; t < N; t++) {
    q[t][8] = (uint32_t)acc[t];
    acc[t] = 0;
  }
#pragma unroll
  for (int c = 0; c < 9; c++) {
#pragma unroll
    for (int j = 0; j <= c; j++) {
      if constexpr (N == 2) {
        mad29x2(acc[0], x[0].v[j], w[0].v[c - j], acc[1], x[1].v[j], w[1].v[c - j]);
        mad29cx2(acc[0], q[0][j], acc[1], q[1][j], Q::RP[c - j]);
      } else {
#pragma unroll
        for (int t = 0; t < N; t++) {
          mad29(acc[t], x[t].v[j], w[t].v[c - j]);
          mad29c(acc[t], q[t][j], Q::RP[c - j]);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < N; t++) {
      out[t].v[c] = (uint32_t)acc[t] & Q::MASK;
      acc[t] >>= 29;
    }
  }
}
NZ_HD F29 mul_shoup(const F29& x, const F29& w, const F29& ws) {
  const F29 xa[1] = {x}, wa[1] = {w}, sa[1] = {ws};
  F29 o[1];
  mul_shoup_n<1>(xa, wa, sa, o);
  return o[0];
}
// two independent Shoup products interleaved (two mad chains side by side, as mul29x2)
NZ_HD void mul_shoup_x2(const F29& x, const F29& w, const F29& ws, const F29& y, const F29& v, const F29& vs, F29& r1,
                        F29& r2) {
  const F29 xa[2] = {x, y}, wa[2] = {w, v}, sa[2] = {ws, vs};
  F29 o[2];
  mul_shoup_n<2>(xa, wa, sa, o);
  r1 = o[0];
  r2 = o[1];
}
// the low 261 bits of a b (normalized a, b)
NZ_HD F29 mul_lo261(const F29& a, const F29& b) {
  F29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int c = 0; c < 9; c++) {
#pragma unroll
    for (int j = 0; j <= c; j++) mad29(acc, a.v[j], b.v[c - j]);
    r.v[c] = (uint32_t)acc & Fr29::MASK;
    acc >>= 29;
  }
  return r;
}

NZ_HD F29 f29_const(const uint32_t (&c)[9]) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = c[i];
  return r;
}

// a * b * 2^-261 mod p (see the invariants above); Q = Fq29 or Fr29
template <class Q = Fq29>
NZ_HD F29 mul29(const F29& a, const F29& b) {
#if NZ_F29_COLS
  return mul29_cols<Q>(a, b);
#endif
  uint32_t m[9];
  F29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) {
      mad29(acc, a.v[j], b.v[i - j]);
      mad29c(acc, m[j], Q::P[i - j]);
    }
    mad29(acc, a.v[i], b.v[0]);
    m[i] = ((uint32_t)acc * Q::INV) & Q::MASK;
    mad29c(acc, m[i], Q::P[0]);
    acc >>= 29;
  }
#pragma unroll
  for (int i = 9; i < 17; i++) {
#pragma unroll
    for (int j = i - 8; j < 9; j++) {
      mad29(acc, a.v[j], b.v[i - j]);
      mad29c(acc, m[j], Q::P[i - j]);
    }
    r.v[i - 9] = (uint32_t)acc & Q::MASK;
    acc >>= 29;
  }
  r.v[8] = (uint32_t)acc;
  return r;
}

// mul29 of two independent products with their instructions interleaved: two dependent
// v_mad_u64_u32 chains side by side, so a wave with few co-resident waves (the NTT's
// 72 KiB-LDS tiles leave 2 per SIMD while the other workgroup loads) keeps issuing
// while one chain waits on its previous mad
template <class Q = Fr29>
NZ_HD void mul29x2(const F29& a, const F29& b, const F29& c, const F29& d, F29& r1, F29& r2) {
#if NZ_F29_COLS
  mul29x2_cols<Q>(a, b, c, d, r1, r2);
#else
  uint32_t m[9], n[9];
  uint64_t acc = 0, bcc = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) {
      mad29x2(acc, a.v[j], b.v[i - j], bcc, c.v[j], d.v[i - j]);
      mad29cx2(acc, m[j], bcc, n[j], Q::P[i - j]);
    }
    mad29x2(acc, a.v[i], b.v[0], bcc, c.v[i], d.v[0]);
    m[i] = ((uint32_t)acc * Q::INV) & Q::MASK;
    n[i] = ((uint32_t)bcc * Q::INV) & Q::MASK;
    mad29cx2(acc, m[i], bcc, n[i], Q::P[0]);
    acc >>= 29;
    bcc >>= 29;
  }
#pragma unroll
  for (int i = 9; i < 17; i++) {
#pragma unroll
    for (int j = i - 8; j < 9; j++) {
      mad29x2(acc, a.v[j], b.v[i - j], bcc, c.v[j], d.v[i - j]);
      mad29cx2(acc, m[j], bcc, n[j], Q::P[i - j]);
    }
    r1.v[i - 9] = (uint32_t)acc & Q::MASK;
    r2.v[i - 9] = (uint32_t)bcc & Q::MASK;
    acc >>= 29;
    bcc >>= 29;
  }
  r1.v[8] = (uint32_t)acc;
  r2.v[8] = (uint32_t)bcc;
#endif
}

// a^2 * 2^-261 mod p: the cross products a_j a_k (j < k) once, against 2 a_k
// (45 instead of 81 product terms; same bounds as mul29, products < 2^59 for
// normalized limbs, so a column stays < 2^64)
NZ_HD F29 sqr29(const F29& a) {
  using Q = Fq29;
  uint32_t a2[9], m[9];
#pragma unroll
  for (int i = 0; i < 9; i++) a2[i] = a.v[i] << 1;
  F29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
#pragma unroll
    for (int j = 0; 2 * j < i; j++) mad29(acc, a.v[j], a2[i - j]);
    if (!(i & 1)) mad29(acc, a.v[i >> 1], a.v[i >> 1]);
#pragma unroll
    for (int j = 0; j < i; j++) mad29c(acc, m[j], Q::P[i - j]);
    m[i] = ((uint32_t)acc * Q::INV) & Q::MASK;
    mad29c(acc, m[i], Q::P[0]);
    acc >>= 29;
  }
#pragma unroll
  for (int i = 9; i < 17; i++) {
#pragma unroll
    for (int j = i - 8; 2 * j < i; j++) mad29(acc, a.v[j], a2[i - j]);
    if (!(i & 1)) mad29(acc, a.v[i >> 1], a.v[i >> 1]);
#pragma unroll
    for (int j = i - 8; j < 9; j++) mad29c(acc, m[j], Q::P[i - j]);
    r.v[i - 9] = (uint32_t)acc & Q::MASK;
    acc >>= 29;
  }
  r.v[8] = (uint32_t)acc;
  return r;
}

// sqr29 of two independent values, interleaved as mul29x2
NZ_HD void sqr29x2(const F29& a, const F29& c, F29& r1, F29& r2) {
#if NZ_F29_COLS
  sqr29x2_cols(a, c, r1, r2);
#else
  using Q = Fq29;
  uint32_t a2[9], c2[9], m[9], n[9];
#pragma unroll
  for (int i = 0; i < 9; i++) {
    a2[i] = a.v[i] << 1;
    c2[i] = c.v[i] << 1;
  }
  uint64_t acc = 0, bcc = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
#pragma unroll
    for (int j = 0; 2 * j < i; j++) mad29x2(acc, a.v[j], a2[i - j], bcc, c.v[j], c2[i - j]);
    if (!(i & 1)) mad29x2(acc, a.v[i >> 1], a.v[i >> 1], bcc, c.v[i >> 1], c.v[i >> 1]);
#pragma unroll
    for (int j = 0; j < i; j++) mad29cx2(acc, m[j], bcc, n[j], Q::P[i - j]);
    m[i] = ((uint32_t)acc * Q::INV) & Q::MASK;
    n[i] = ((uint32_t)bcc * Q::INV) & Q::MASK;
    mad29cx2(acc, m[i], bcc, n[i], Q::P[0]);
    acc >>= 29;
    bcc >>= 29;
  }
#pragma unroll
  for (int i = 9; i < 17; i++) {
#pragma unroll
    for (int j = i - 8; 2 * j < i; j++) mad29x2(acc, a.v[j], a2[i - j], bcc, c.v[j], c2[i - j]);
    if (!(i & 1)) mad29x2(acc, a.v[i >> 1], a.v[i >> 1], bcc, c.v[i >> 1], c.v[i >> 1]);
#pragma unroll
    for (int j = i - 8; j < 9; j++) mad29cx2(acc, m[j], bcc, n[j], Q::P[i - j]);
    r1.v[i - 9] = (uint32_t)acc & Q::MASK;
    r2.v[i - 9] = (uint32_t)bcc & Q::MASK;
    acc >>= 29;
    bcc >>= 29;
  }
  r1.v[8] = (uint32_t)acc;
  r2.v[8] = (uint32_t)bcc;
#endif
}

// (a b + c d) * 2^-261 mod p with one Montgomery reduction. Needs every limb < 2^29
// (normalized or product outputs: a column is <= 27 terms < 2^58) and a, b, c, d < 2^257
// with a b + c d < 2^515; result < 2p for the operand sizes used (see msm.hip)
NZ_HD F29 mul2sum29(const F29& a, const F29& b, const F29& c, const F29& d) {
#if NZ_F29_COLS
  return mul2sum29_cols(a, b, c, d);
#else
  using Q = Fq29;
  uint32_t m[9];
  F29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
#pragma unroll
    for (int j = 0; j <= i; j++) {
      mad29(acc, a.v[j], b.v[i - j]);
      mad29(acc, c.v[j], d.v[i - j]);
    }
#pragma unroll
    for (int j = 0; j < i; j++) mad29c(acc, m[j], Q::P[i - j]);
    m[i] = ((uint32_t)acc * Q::INV) & Q::MASK;
    mad29c(acc, m[i], Q::P[0]);
    acc >>= 29;
  }
#pragma unroll
  for (int i = 9; i < 17; i++) {
#pragma unroll
    for (int j = i - 8; j < 9; j++) {
      mad29(acc, a.v[j], b.v[i - j]);
      mad29(acc, c.v[j], d.v[i - j]);
      mad29c(acc, m[j], Q::P[i - j]);
    }
    r.v[i - 9] = (uint32_t)acc & Q::MASK;
    acc >>= 29;
  }
  r.v[8] = (uint32_t)acc;
  return r;
#endif
}

// sum_k a[k] b[k] * 2^-261 mod q with one Montgomery reduction (K <= 6 keeps a column
// of 9K + 9 terms < 2^58 below 2^64). Needs normalized limbs (< 2^29); for inputs
// below 4q the result is below (0.1 K + 1) q < 2q for K <= 6 (q ~ 2^253.6).
template <class Q, int K>
NZ_HD F29 mulsum29(const F29 (&a)[K], const F29 (&b)[K]) {
#if NZ_F29_COLS
  if constexpr (K == 2) return mulsum29_cols2<Q>(a, b);
  if constexpr (K == 3) return mulsum29_cols3<Q>(a, b);
  if constexpr (K == 4) return mulsum29_cols4<Q>(a, b);
  if constexpr (K == 5) return mulsum29_cols5<Q>(a, b);
  if constexpr (K == 6) return mulsum29_cols6<Q>(a, b);
#endif
  uint32_t m[9];
  F29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
#pragma unroll
    for (int k = 0; k < K; k++)
#pragma unroll
      for (int j = 0; j <= i; j++) mad29(acc, a[k].v[j], b[k].v[i - j]);
#pragma unroll
    for (int j = 0; j < i; j++) mad29c(acc, m[j], Q::P[i - j]);
    m[i] = ((uint32_t)acc * Q::INV) & Q::MASK;
    mad29c(acc, m[i], Q::P[0]);
    acc >>= 29;
  }
#pragma unroll
  for (int i = 9; i < 17; i++) {
#pragma unroll
    for (int j = i - 8; j < 9; j++) {
#pragma unroll
      for (int k = 0; k < K; k++) mad29(acc, a[k].v[j], b[k].v[i - j]);
      mad29c(acc, m[j], Q::P[i - j]);
    }
    r.v[i - 9] = (uint32_t)acc & Q::MASK;
    acc >>= 29;
  }
  r.v[8] = (uint32_t)acc;
  return r;
}

NZ_HD void norm29(F29& r) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r.v[i + 1] += r.v[i] >> 29;
    r.v[i] &= Fq29::MASK;
  }
}

// a + K - b, normalized (K borrowed-form multiple of p, b < K)
NZ_HD F29 sub29(const F29& a, const F29& b, const uint32_t (&K)[9]) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = a.v[i] + K[i] - b.v[i];
  norm29(r);
  return r;
}

// a + b (+ b again when twice), normalized
NZ_HD F29 add29(const F29& a, const F29& b) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = a.v[i] + b.v[i];
  norm29(r);
  return r;
}
NZ_HD F29 add2x29(const F29& a, const F29& b) {  // a + 2b
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = a.v[i] + (b.v[i] << 1);
  norm29(r);
  return r;
}

// Unnormalized forms for operands whose next use tolerates wider limbs. mul29 and
// mul2sum29 accept one factor of each product with limbs < 2^31 when the other factor is
// normalized: a column then stays below 9 (2^60.5 + 2^58) + 2^35 < 2^64 (mul29) and
// 9 (2^59.6 + 2^59 + 2^58) + 2^35 < 2^64 (mul2sum29 with b < 2^30.6, c < 2^30). Saves the
// 24-instruction carry normalisation where the value feeds a product next. Every limb,
// the top one included, must stay non-negative: K's top limb must exceed b's.
// a + K - b with K borrowed (limbs >= 2^29 - 1), a, b normalized: limbs < 2^29 + K_i
NZ_HD F29 sub29_nn(const F29& a, const F29& b, const uint32_t (&K)[9]) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = a.v[i] + K[i] - b.v[i];
  return r;
}
// 4p - y for a normalized y < 2p (a product output): limbs < 2^30
NZ_HD F29 neg4p29_nn(const F29& y) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = Fq29::K4[i] - y.v[i];
  return r;
}
// 2p - y for a normalized y <= p: limbs < 2^30. (p - y would leave the top limb at -1
// when y's top limb equals p's: the borrowed form needs the next multiple.)
NZ_HD F29 neg29_nn(const F29& y) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = Fq29::K2[i] - y.v[i];
  return r;
}
// a + 6p - b - 2c for normalized a, b, c with b, c < 2p, normalized: 6p in a wide borrowed
// form (limbs 0..7 in [2^31 - 4, 2^31 + 2^29), so a limb never goes negative and never
// passes 2^32; the top limb may wrap, the normalised value a + 6p - b - 2c >= 0 is exact)
struct Fq29W {
  // 10p borrowed (limbs 0..7 in [2^29 - 1, 2^30)): Q - X3 + 10p for X3 < 8p keeps every
  // limb, the top one included, non-negative (8p's top limb would not)
  static constexpr uint32_t K10[9] = {0x34e1e4c6u, 0x2a2bc722u, 0x3c7a6115u, 0x3c535c27u, 0x373a7eafu,
                                      0x3c908785u, 0x2684cc89u, 0x2f997e07u, 0x01e3eb0fu};
  static constexpr uint32_t K6W[9] = {0x92edefaau, 0x861a4444u, 0x8aafd3d6u, 0x90fed0e1u, 0x812318ccu,
                                      0x91238480u, 0x83e94782u, 0x9628e534u, 0x012259d2u};
};
NZ_HD F29 sub2x29(const F29& a, const F29& b, const F29& c) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = a.v[i] + Fq29W::K6W[i] - b.v[i] - (c.v[i] << 1);
  norm29(r);
  return r;
}

// 4p - y for y < 4p (K4 borrowed form), normalized
NZ_HD F29 neg4p29(const F29& y) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = Fq29::K4[i] - y.v[i];
  norm29(r);
  return r;
}

// p - y for a normalized y <= p (negated base ordinate), normalized
NZ_HD F29 neg29(const F29& y) {
  F29 r;
  r.v[0] = Fq29::P[0] + (1u << 29) - y.v[0];
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = Fq29::P[i] + (1u << 29) - 1u - y.v[i];
  r.v[8] = Fq29::P[8] - 1u - y.v[8];
  norm29(r);
  return r;
}

// x == 0 mod p for a product output (normalized, < 2p): x is 0 or p
NZ_HD bool is0p29(const F29& x) {
  uint32_t o0 = 0, op = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    o0 |= x.v[i];
    op |= x.v[i] ^ Fq29::P[i];
  }
  return o0 == 0 || op == 0;
}

// is0p29 for a product output, with a one-limb early exit (a nonzero product almost
// never has a low limb of 0 or p's; the full test runs only then)
NZ_HD bool is0p29_fast(const F29& x) {
  if (x.v[0] != 0u && x.v[0] != Fq29::P[0]) return false;
  return is0p29(x);
}

// radix change of the same integer (< 2^256, no Montgomery change)
template <class Par>
NZ_HD F29 split29(const Fe<Par>& x) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int bit = 29 * i, limb = bit >> 5, sh = bit & 31;
    uint64_t w = x.v[limb];
    if (limb + 1 < 8) w |= (uint64_t)x.v[limb + 1] << 32;
    r.v[i] = (uint32_t)(w >> sh) & Fq29::MASK;
  }
  return r;
}
NZ_HD Fq join29(const F29& x) {  // x normalized, < 2^256
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int bit = 29 * i, limb = bit >> 5, sh = bit & 31;
    const uint64_t w = (uint64_t)x.v[i] << sh;
    r.v[limb] |= (uint32_t)w;
    if (limb + 1 < 8) r.v[limb + 1] |= (uint32_t)(w >> 32);
  }
  return r;
}

// a * w for a canonical Montgomery-256 Fr and a twiddle w given as split29 of its
// Montgomery-261 form (w * 2^261 mod r): one 9x29 product instead of the 8x32 mac
// chain of field.h, canonical Montgomery-256 result
// normalized F29 below 2r -> canonical Fr (same integer mod r, no Montgomery change)
NZ_HD Fr join_fr29(const F29& t) {
  Fr r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int bit = 29 * i, limb = bit >> 5, sh = bit & 31;
    const uint64_t w = (uint64_t)t.v[i] << sh;
    r.v[limb] |= (uint32_t)w;
    if (limb + 1 < 8) r.v[limb + 1] |= (uint32_t)(w >> 32);
  }
  return reduce_once(r);
}
// normalized x < 128 r -> canonical Fr: q = floor(x_8 / (r_8 + 1)) <= x / r, x - q r < 2r
// (ntt.hip's last pass, round 5's k_pol_r / k_pol_wxi)
NZ_HD Fr canon_fr29(const F29& x) {
  const uint32_t q = x.v[8] / (Fr29::P[8] + 1u);
  F29 y;
  int64_t carry = 0;
#pragma unroll
  for (int l = 0; l < 9; l++) {
    const int64_t t = (int64_t)x.v[l] + carry - (int64_t)((uint64_t)q * Fr29::P[l]);
    y.v[l] = l < 8 ? ((uint32_t)t & Fr29::MASK) : (uint32_t)t;
    carry = t >> 29;
  }
  return join_fr29(y);
}
NZ_HD Fr mul_fr29(const Fr& a, const F29& w29) {
  return join_fr29(mul29<Fr29>(split29(a), w29));  // product < 2r, limbs < 2^29
}

// a * 2^-256 mod r: Montgomery-256 Fr -> canonical normal form (the MSM's scalars), as
// mul29<Fr29>(split29(a), 32) with the single-term product columns a_i * 32 (81
// reduction mads instead of field.h's 8x32 product by 1)
NZ_HD Fr from_mont_fr29(const Fr& a) {
  using Q = Fr29;
  const F29 x = split29(a);
  uint32_t m[9];
  F29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    acc += (uint64_t)x.v[i] << 5;
#pragma unroll
    for (int j = 0; j < i; j++) mad29c(acc, m[j], Q::P[i - j]);
    m[i] = ((uint32_t)acc * Q::INV) & Q::MASK;
    mad29c(acc, m[i], Q::P[0]);
    acc >>= 29;
  }
#pragma unroll
  for (int i = 9; i < 17; i++) {
#pragma unroll
    for (int j = i - 8; j < 9; j++) mad29c(acc, m[j], Q::P[i - j]);
    r.v[i - 9] = (uint32_t)acc & Q::MASK;
    acc >>= 29;
  }
  r.v[8] = (uint32_t)acc;
  return join_fr29(r);
}

// Montgomery-256 Fr -> the same value at exponent 261 (x 2^5 < 32 r, normalized): the
// 261-bit shift of the limbs, no product (x < 2^254, so the top limb stays < 2^27)
NZ_HD F29 fr_to261(const Fr& x) {
  const F29 r = split29(x);
  F29 o;
  o.v[0] = (r.v[0] << 5) & Fr29::MASK;
#pragma unroll
  for (int l = 1; l < 9; l++) o.v[l] = ((r.v[l] << 5) & Fr29::MASK) | (r.v[l - 1] >> 24);
  return o;
}
NZ_HD F29 add3_29(const F29& a, const F29& b, const F29& c) {  // normalized
  F29 r;
#pragma unroll
  for (int l = 0; l < 9; l++) r.v[l] = a.v[l] + b.v[l] + c.v[l];
  norm29(r);
  return r;
}
// exponent 261 -> canonical Montgomery-256 Fr (one product by 2^256 mod r)
NZ_HD Fr fr_from261(const F29& x) { return join_fr29(mul29<Fr29>(x, f29_const(Fr29::C256))); }

// Montgomery-261 value (any F29 < 2^257) -> canonical Montgomery-256 Fq (csrc/field.h)
NZ_HD Fq to_fq256(const F29& x) { return reduce_once(join29(mul29(x, f29_const(Fq29::C256)))); }

// XYZZ point with Montgomery-261 coordinates: X < 8p, Y < 4p, ZZ, ZZZ < 2p.
// Stored as 144 bytes; infinity is stored with ZZ = 0 (a finite point's ZZ is never
// 0 or p).
struct alignas(16) Xyzz29 {
  F29 X, Y, ZZ, ZZZ;
};

// doubling of an affine point (x, y < p+1, normalized): dbl-2008-s-1 with Z = 1
NZ_HD Xyzz29 mdbl29(const F29& x, const F29& y) {
  Xyzz29 r;
  F29 U;
#pragma unroll
  for (int i = 0; i < 9; i++) U.v[i] = y.v[i] << 1;  // < 2p, limbs < 2^30
  const F29 V = sqr29(U);
  const F29 W = mul29(U, V);
  const F29 S = mul29(x, V);
  const F29 xx = sqr29(x);
  F29 M;
#pragma unroll
  for (int i = 0; i < 9; i++) M.v[i] = xx.v[i] * 3u;  // < 6p
  norm29(M);
  const F29 t = add29(S, S);                                      // < 4p
  r.X = sub29(sqr29(M), t, Fq29::K4);                          // < 6p
  const F29 d = sub29(S, r.X, Fq29::K8);                          // < 10p
  r.Y = sub29(mul29(M, d), mul29(W, y), Fq29::K2);                // < 4p
  r.ZZ = V;
  r.ZZZ = W;
  return r;
}

NZ_HD bool is_inf29(const Xyzz29& a) {
  uint32_t z = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) z |= a.ZZ.v[i];
  return z == 0;
}

// dbl-2008-s-1 (a = 0) of a finite XYZZ point (its Y is never 0 mod p on BN254 G1)
NZ_HD Xyzz29 dbl29(const Xyzz29& p) {
  Xyzz29 r;
  F29 U;
#pragma unroll
  for (int i = 0; i < 9; i++) U.v[i] = p.Y.v[i] << 1;  // < 8p, limbs < 2^30
  const F29 V = sqr29(U);
  const F29 W = mul29(U, V);
  const F29 S = mul29(p.X, V);
  const F29 xx = sqr29(p.X);
  F29 M;
#pragma unroll
  for (int i = 0; i < 9; i++) M.v[i] = xx.v[i] * 3u;  // < 6p
  norm29(M);
  r.X = sub29(sqr29(M), add29(S, S), Fq29::K4);   // < 6p
  r.Y = sub29(mul29(M, sub29(S, r.X, Fq29::K8)), mul29(W, p.Y), Fq29::K2);  // < 4p
  r.ZZ = mul29(V, p.ZZ);
  r.ZZZ = mul29(W, p.ZZZ);
  return r;
}

// add-2008-s: XYZZ + XYZZ (infinity = ZZ stored as 0), 12 products + 2 squares. The
// independent products run in interleaved pairs (mul29x2 / sqr29x2: U1 | U2, S1 | S2,
// PP | RR, PPP | Q, ZZ1 ZZ2 | ZZZ1 ZZZ2, ZZ3 | ZZZ3, and Y3's two terms): seven dependent
// product steps instead of fourteen, which is what the bucket reduction's trees wait on
NZ_HD Xyzz29 add29(const Xyzz29& p, const Xyzz29& q) {
  if (is_inf29(p)) return q;
  if (is_inf29(q)) return p;
  F29 U1, U2, S1, S2, PP, RR, PPP, Q, Z12, ZZZ12;
  mul29x2<Fq29>(p.X, q.ZZ, q.X, p.ZZ, U1, U2);
  mul29x2<Fq29>(p.Y, q.ZZZ, q.Y, p.ZZZ, S1, S2);
  const F29 P = sub29(U2, U1, Fq29::K2);  // < 4p
  const F29 R = sub29(S2, S1, Fq29::K2);  // < 4p
  sqr29x2(P, R, PP, RR);
  mul29x2<Fq29>(P, PP, U1, PP, PPP, Q);
  mul29x2<Fq29>(p.ZZ, q.ZZ, p.ZZZ, q.ZZZ, Z12, ZZZ12);
  Xyzz29 r;
  mul29x2<Fq29>(Z12, PP, ZZZ12, PPP, r.ZZ, r.ZZZ);
  if (is0p29(r.ZZ)) {  // same abscissa
    if (is0p29(RR)) return dbl29(p);
    Xyzz29 inf = r;
#pragma unroll
    for (int i = 0; i < 9; i++) inf.ZZ.v[i] = 0;
    return inf;
  }
  r.X = sub29(RR, add2x29(PPP, Q), Fq29::K6);  // < 8p
  F29 y1, y2;
  mul29x2<Fq29>(R, sub29(Q, r.X, Fq29::K8), S1, PPP, y1, y2);
  r.Y = sub29(y1, y2, Fq29::K2);  // < 4p
  return r;
}

}  // namespace nzcb
