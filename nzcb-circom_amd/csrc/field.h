// BN254 Fq / Fr Montgomery arithmetic on 8 x 32-bit limbs, for gfx950 wavefronts.
//
// Replaces the field layer the reference reaches through
// snarkjs@0.4.12 -> ffjavascript@0.2.48 -> wasmcurves@0.1.0 (f1m_* / frm_*;
// /root/reference/yarn.lock:3905-3913, 8173-8179).
// Representation matches the zkey's "LEM" bytes exactly: little-endian limbs of
// x * 2^256 mod m, so zkey sections are uploaded to HBM without conversion.
//
// One lane owns one element (no cross-lane limb splitting): every hot kernel on
// this path is element-parallel (NTT butterflies, bucket adds, pointwise rounds),
// so 64 independent multiplies per wavefront keep the VALU busy without shuffles.
// Multiplication is product-scanning Montgomery (Koc's FIPS ordering) with a
// 96-bit column accumulator: each 32x32 partial product is one v_mad_u64_u32
// plus one carry add, and no intermediate t[] array is kept live.
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define NZ_HD __host__ __device__ __forceinline__
#else
#define NZ_HD inline
#endif

namespace nzcb {

struct FqParams {
  static constexpr uint32_t P[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                    0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr uint32_t INV = 0xe4866389u;  // -p^-1 mod 2^32
  static constexpr uint64_t INV64 = 0x87d20782e4866389ULL;
  static constexpr uint32_t ONE[8] = {0xc58f0d9du, 0xd35d438du, 0xf5c70b3du, 0x0a78eb28u,
                                      0x7879462cu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
  static constexpr uint32_t R2[8] = {0x538afa89u, 0xf32cfc5bu, 0xd44501fbu, 0xb5e71911u,
                                     0x0a417ff6u, 0x47ab1effu, 0xcab8351fu, 0x06d89f71u};
};

struct FrParams {
  static constexpr uint32_t P[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                                    0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr uint32_t INV = 0xefffffffu;
  static constexpr uint64_t INV64 = 0xc2e1f593efffffffULL;
  static constexpr uint32_t ONE[8] = {0x4ffffffbu, 0xac96341cu, 0x9f60cd29u, 0x36fc7695u,
                                      0x7879462eu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
  static constexpr uint32_t R2[8] = {0xae216da7u, 0x1bb8e645u, 0xe35c59e3u, 0x53fe3ab1u,
                                     0x53bb8085u, 0x8c49833du, 0x7f4e44a5u, 0x0216d0b1u};
};

template <class Par>
struct alignas(16) Fe {
  uint32_t v[8];

  NZ_HD static Fe zero() {
    Fe r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = 0;
    return r;
  }
  NZ_HD static Fe one() {
    Fe r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = Par::ONE[i];
    return r;
  }
  NZ_HD static Fe r2() {
    Fe r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = Par::R2[i];
    return r;
  }
  NZ_HD static Fe modulus() {
    Fe r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = Par::P[i];
    return r;
  }
  NZ_HD bool is_zero() const {
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x |= v[i];
    return x == 0;
  }
  NZ_HD bool operator==(const Fe& o) const {
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x |= v[i] ^ o.v[i];
    return x == 0;
  }
  NZ_HD bool operator!=(const Fe& o) const { return !(*this == o); }
};

using Fq = Fe<FqParams>;
using Fr = Fe<FrParams>;

// ---- limb helpers -----------------------------------------------------------
// Carry chains through clang's add/sub-with-carry builtins: on gfx950 they lower to
// one v_add_co / v_addc_co (v_sub_co / v_subb_co) per limb. The 64-bit C form
// ((uint64_t)a + b + carry) became two v_lshl_add_u64 plus zero-extension moves per
// limb (about 5 instructions), and field additions were a third of an NTT pass.
NZ_HD uint32_t addc(uint32_t a, uint32_t b, uint32_t& carry) {
  unsigned int c;
  const uint32_t s = __builtin_addc(a, b, carry, &c);
  carry = c;
  return s;
}
NZ_HD uint32_t subb(uint32_t a, uint32_t b, uint32_t& borrow) {
  unsigned int c;
  const uint32_t d = __builtin_subc(a, b, borrow, &c);
  borrow = c;
  return d;
}

// r = a - p if a >= p else a   (a < 2p)
template <class Par>
NZ_HD Fe<Par> reduce_once(const Fe<Par>& a) {
  Fe<Par> t;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) t.v[i] = subb(a.v[i], Par::P[i], br);
  Fe<Par> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = br ? a.v[i] : t.v[i];
  return r;
}

template <class Par>
NZ_HD Fe<Par> operator+(const Fe<Par>& a, const Fe<Par>& b) {
  Fe<Par> s;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s.v[i] = addc(a.v[i], b.v[i], c);
  return reduce_once(s);
}

template <class Par>
NZ_HD Fe<Par> operator-(const Fe<Par>& a, const Fe<Par>& b) {
  Fe<Par> d;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d.v[i] = subb(a.v[i], b.v[i], br);
  // add back p when the subtraction borrowed (mask form keeps it branch-free)
  uint32_t mask = 0u - br;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d.v[i] = addc(d.v[i], Par::P[i] & mask, c);
  return d;
}

template <class Par>
NZ_HD Fe<Par> neg(const Fe<Par>& a) {
  return Fe<Par>::zero() - a;
}

template <class Par>
NZ_HD Fe<Par> dbl(const Fe<Par>& a) {
  return a + a;
}

// 96-bit column accumulator step: (hi:acc) += x*y.
// On gfx950 this is v_mad_u64_u32 with its carry-out in an SGPR pair, folded into
// `hi` by v_addc_co_u32. A VALU write of an SGPR consumed as a carry-in needs two
// wait states (hipcc inserts the same s_nop for its own v_cmp/v_addc pairs), hence
// the s_nop 1. Measured on MI355X: 106 G mont-mul/s vs 61 G for the plain C form
// (nzcb-circom_amd/tools/mulbench.hip), bit-identical results.
// Variants (A/B'd on the full n=2^21 proof, tools/variant_bench.py, MI355X):
//   0 asm volatile            10.9 proofs/s   (volatile pins every mac in program order)
//   1 asm, schedulable        13.4 proofs/s   <- default: independent products interleave
//   2 plain C (v_cmp carry)   10.9 proofs/s
//   3 asm, two column chains  12.6 proofs/s
#ifndef NZ_MAC_VARIANT
#define NZ_MAC_VARIANT 1
#endif
#if NZ_MAC_VARIANT == 0
#define NZ_MAC_ASM asm volatile
#else
#define NZ_MAC_ASM asm
#endif
#if defined(__HIP_DEVICE_COMPILE__) && NZ_MAC_VARIANT != 2
__device__ __forceinline__ void mac(uint64_t& acc, uint32_t& hi, uint32_t x, uint32_t y) {
  uint64_t c;
  NZ_MAC_ASM("v_mad_u64_u32 %0, %1, %3, %4, %0\n\ts_nop 1\n\tv_addc_co_u32_e64 %2, %1, %2, 0, %1"
             : "+v"(acc), "=&s"(c), "+v"(hi)
             : "v"(x), "v"(y));
}
// same with y a wave-uniform constant (modulus limb) held in an SGPR
__device__ __forceinline__ void mac_c(uint64_t& acc, uint32_t& hi, uint32_t x, uint32_t y) {
  uint64_t c;
  NZ_MAC_ASM("v_mad_u64_u32 %0, %1, %3, %4, %0\n\ts_nop 1\n\tv_addc_co_u32_e64 %2, %1, %2, 0, %1"
             : "+v"(acc), "=&s"(c), "+v"(hi)
             : "v"(x), "s"(y));
}
#else
NZ_HD void mac(uint64_t& acc, uint32_t& hi, uint32_t x, uint32_t y) {
  uint64_t t = (uint64_t)x * y + acc;
  hi += (t < acc) ? 1u : 0u;
  acc = t;
}
NZ_HD void mac_c(uint64_t& acc, uint32_t& hi, uint32_t x, uint32_t y) { mac(acc, hi, x, y); }
#endif

#if !defined(__HIP_DEVICE_COMPILE__)
// Host: 4 x 64-bit CIOS with 128-bit products (transcript scalars, window folds).
template <class Par>
inline Fe<Par> mont_mul_host(const Fe<Par>& a, const Fe<Par>& b) {
  typedef unsigned __int128 u128;
  uint64_t A[4], Bv[4], P[4];
  memcpy(A, a.v, 32);
  memcpy(Bv, b.v, 32);
  memcpy(P, Par::P, 32);
  const uint64_t inv = (uint64_t)Par::INV64;
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c += (u128)A[j] * Bv[i] + t[j];
      t[j] = (uint64_t)c;
      c >>= 64;
    }
    c += t[4];
    t[4] = (uint64_t)c;
    t[5] = (uint64_t)(c >> 64);
    uint64_t m = t[0] * inv;
    c = (u128)m * P[0] + t[0];
    c >>= 64;
    for (int j = 1; j < 4; j++) {
      c += (u128)m * P[j] + t[j];
      t[j - 1] = (uint64_t)c;
      c >>= 64;
    }
    c += t[4];
    t[3] = (uint64_t)c;
    t[4] = t[5] + (uint64_t)(c >> 64);
  }
  Fe<Par> r;
  memcpy(r.v, t, 32);
  return reduce_once(r);
}
#endif

// Montgomery product a*b*2^-256 mod m, inputs < m, output < m.
template <class Par>
NZ_HD Fe<Par> operator*(const Fe<Par>& a, const Fe<Par>& b) {
#if !defined(__HIP_DEVICE_COMPILE__)
  return mont_mul_host(a, b);
#endif
#if NZ_MAC_VARIANT == 3
  // two independent column chains (a*b terms, m*p terms) merged once per column:
  // halves the dependent v_mad_u64_u32 chain a wave has to wait on
  uint32_t m[8];
  Fe<Par> r;
  uint64_t acc = 0, acc2 = 0;
  uint32_t hi = 0, hi2 = 0;
  auto merge = [&]() {
    uint64_t s = acc + acc2;
    hi += hi2 + (s < acc ? 1u : 0u);
    acc = s;
    acc2 = 0;
    hi2 = 0;
  };
#pragma unroll
  for (int i = 0; i < 8; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) {
      mac(acc, hi, a.v[j], b.v[i - j]);
      mac_c(acc2, hi2, m[j], Par::P[i - j]);
    }
    mac(acc, hi, a.v[i], b.v[0]);
    merge();
    m[i] = (uint32_t)acc * Par::INV;
    mac_c(acc, hi, m[i], Par::P[0]);
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
#pragma unroll
  for (int i = 8; i < 15; i++) {
#pragma unroll
    for (int j = i - 7; j < 8; j++) {
      mac(acc, hi, a.v[j], b.v[i - j]);
      mac_c(acc2, hi2, m[j], Par::P[i - j]);
    }
    merge();
    r.v[i - 8] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  r.v[7] = (uint32_t)acc;
  return reduce_once(r);
#else
  uint32_t m[8];
  Fe<Par> r;
  uint64_t acc = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) {
      mac(acc, hi, a.v[j], b.v[i - j]);
      mac_c(acc, hi, m[j], Par::P[i - j]);
    }
    mac(acc, hi, a.v[i], b.v[0]);
    m[i] = (uint32_t)acc * Par::INV;
    mac_c(acc, hi, m[i], Par::P[0]);
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
#pragma unroll
  for (int i = 8; i < 15; i++) {
#pragma unroll
    for (int j = i - 7; j < 8; j++) {
      mac(acc, hi, a.v[j], b.v[i - j]);
      mac_c(acc, hi, m[j], Par::P[i - j]);
    }
    r.v[i - 8] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  r.v[7] = (uint32_t)acc;  // < 2m < 2^256, so the top word is empty
  return reduce_once(r);
#endif
}

template <class Par>
NZ_HD Fe<Par> sqr(const Fe<Par>& a) {
  return a * a;
}

template <class Par>
NZ_HD Fe<Par> to_mont(const Fe<Par>& a) {
  return a * Fe<Par>::r2();
}

template <class Par>
NZ_HD Fe<Par> from_mont(const Fe<Par>& a) {
  Fe<Par> one_n = Fe<Par>::zero();
  one_n.v[0] = 1;
  return a * one_n;
}

// a^e for a 256-bit exponent given as 8 limbs (square-and-multiply, MSB first)
template <class Par>
NZ_HD Fe<Par> pow_limbs(const Fe<Par>& a, const uint32_t e[8]) {
  Fe<Par> r = Fe<Par>::one();
  bool started = false;
  for (int i = 7; i >= 0; i--) {
    for (int b = 31; b >= 0; b--) {
      if (started) r = sqr(r);
      if ((e[i] >> b) & 1u) {
        r = started ? r * a : a;
        started = true;
      }
    }
  }
  return r;
}

template <class Par>
NZ_HD Fe<Par> pow_u64(const Fe<Par>& a, uint64_t e) {
  Fe<Par> r = Fe<Par>::one();
  Fe<Par> b = a;
  while (e) {
    if (e & 1) r = r * b;
    b = sqr(b);
    e >>= 1;
  }
  return r;
}

// Fermat inverse a^(m-2); inverse of zero returns zero.
template <class Par>
NZ_HD Fe<Par> inverse(const Fe<Par>& a) {
  uint32_t e[8];
  uint32_t br = 0;
  e[0] = subb(Par::P[0], 2u, br);
#pragma unroll
  for (int i = 1; i < 8; i++) e[i] = subb(Par::P[i], 0u, br);
  return pow_limbs(a, e);
}

}  // namespace nzcb
