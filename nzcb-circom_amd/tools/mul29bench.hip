// Microbenchmark: Montgomery product in a redundant 9 x 29-bit radix (R = 2^261) vs the
// 8 x 32-bit product-scanning product of csrc/field.h, on gfx950.
//
// With 29-bit limbs every partial product is < 2^58 (< 2^60 with one bit of limb slack),
// so a whole column (<= 18 products) fits one 64-bit accumulator: each partial product is
// ONE v_mad_u64_u32 and no carry instruction, against mad + addc (2 x 4 cycles) at 32 bits.
// Inputs may be any value < 2^257 with limbs < 2^30; the output is < 2p, limbs < 2^29.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../csrc/field.h"
using namespace nzcb;

struct F29 {
  uint32_t v[9];
};
static constexpr uint32_t kInv29 = 0x04866389u;
static constexpr uint32_t kMask29 = (1u << 29) - 1;

__device__ __forceinline__ F29 mul29(const F29& a, const F29& b) {
  constexpr uint32_t P[9] = {0x187cfd47u, 0x010460b6u, 0x1c72a34fu, 0x02d522d0u, 0x1585d978u,
                             0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
  uint32_t m[9];
  F29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) {
      acc += (uint64_t)a.v[j] * b.v[i - j];
      acc += (uint64_t)m[j] * P[i - j];
    }
    acc += (uint64_t)a.v[i] * b.v[0];
    m[i] = ((uint32_t)acc * kInv29) & kMask29;
    acc += (uint64_t)m[i] * P[0];
    acc >>= 29;
  }
#pragma unroll
  for (int i = 9; i < 17; i++) {
#pragma unroll
    for (int j = i - 8; j < 9; j++) {
      acc += (uint64_t)a.v[j] * b.v[i - j];
      acc += (uint64_t)m[j] * P[i - j];
    }
    r.v[i - 9] = (uint32_t)acc & kMask29;
    acc >>= 29;
  }
  r.v[8] = (uint32_t)acc;
  return r;
}

// radix conversion of the same integer (no Montgomery change)
__host__ __device__ inline F29 split29(const Fq& x) {
  F29 r;
  for (int i = 0; i < 9; i++) {
    const int bit = 29 * i, limb = bit >> 5, sh = bit & 31;
    uint64_t w = x.v[limb];
    if (limb + 1 < 8) w |= (uint64_t)x.v[limb + 1] << 32;
    r.v[i] = (uint32_t)(w >> sh) & kMask29;
  }
  return r;
}
__host__ __device__ inline Fq join29(const F29& x) {  // x < 2^256, normalized limbs
  Fq r;
  for (int i = 0; i < 8; i++) r.v[i] = 0;
  for (int i = 0; i < 9; i++) {
    const int bit = 29 * i, limb = bit >> 5, sh = bit & 31;
    uint64_t w = (uint64_t)x.v[i] << sh;
    r.v[limb] |= (uint32_t)w;
    if (limb + 1 < 8) r.v[limb + 1] |= (uint32_t)(w >> 32);
  }
  return r;
}

template <int V>
__global__ void chain(Fq* io, int iters) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (V == 0) {
    Fq a = io[2 * i], b = io[2 * i + 1];
    for (int k = 0; k < iters; k++) {
      a = a * b;
      b = b * a;
    }
    io[2 * i] = a;
    io[2 * i + 1] = b;
  } else {
    F29 a = split29(io[2 * i]), b = split29(io[2 * i + 1]);
    for (int k = 0; k < iters; k++) {
      a = mul29(a, b);
      b = mul29(b, a);
    }
    io[2 * i] = join29(a);
    io[2 * i + 1] = join29(b);
  }
}

// correctness: mont29(a,b) * 2^5 == mont32(a,b)  (both reduced mod p); k = 2^261 mod p (normal)
__global__ void check(const Fq* in, const Fq k261, int n, int* bad) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fq a = in[2 * i], b = in[2 * i + 1];
  Fq want = a * b;  // a*b*2^-256
  Fq r = reduce_once(join29(mul29(split29(a), split29(b))));  // a*b*2^-261 (< 2p -> < p)
  Fq got = r * k261;  // * 2^261 * 2^-256 = a*b*2^-256
  if (!(got == want)) atomicAdd(bad, 1);
  // chained: outputs (< 2p, unreduced) fed back as inputs
  F29 x = mul29(split29(a), split29(b));
  F29 y = mul29(x, x);
  Fq yr = reduce_once(join29(y));
  Fq xr = r;                              // x reduced, in the 2^-261 domain
  Fq w = xr * xr;                         // x*x*2^-256
  Fq y2 = yr * k261;                      // x*x*2^-261 * 2^261 * 2^-256
  if (!(w == y2)) atomicAdd(bad, 1);
}

int main() {
  const int blocks = 256 * 16, threads = 256, iters = 200;
  size_t n = (size_t)blocks * threads;
  Fq* d;
  (void)hipMalloc(&d, n * 2 * sizeof(Fq));
  Fq* h = (Fq*)malloc(n * 2 * sizeof(Fq));
  srand(1);
  for (size_t i = 0; i < 2 * n; i++) {
    for (int j = 0; j < 8; j++) h[i].v[j] = rand() ^ (rand() << 16);
    h[i].v[7] &= 0x0fffffff;
  }
  // k261 = 2^261 mod p as a plain integer: to_mont(32) = 32 * 2^256 mod p
  Fq thirty_two = Fq::zero();
  thirty_two.v[0] = 32;
  const Fq k261 = to_mont(thirty_two);
  int* dbad;
  (void)hipMalloc(&dbad, 4);
  (void)hipMemset(dbad, 0, 4);
  (void)hipMemcpy(d, h, n * 2 * sizeof(Fq), hipMemcpyHostToDevice);
  check<<<(1 << 16) / 256, 256>>>(d, k261, 1 << 16, dbad);
  int bad = 0;
  (void)hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost);
  printf("mul29 correctness: %s (%d mismatches of %d)\n", bad ? "MISMATCH" : "ok", bad, 2 << 16);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int v = 0; v < 2; v++) {
    (void)hipMemcpy(d, h, n * 2 * sizeof(Fq), hipMemcpyHostToDevice);
    if (v == 0) chain<0><<<blocks, threads>>>(d, 2);
    else chain<1><<<blocks, threads>>>(d, 2);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    if (v == 0) chain<0><<<blocks, threads>>>(d, iters);
    else chain<1><<<blocks, threads>>>(d, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%s: %.3f ms, %.1f G mont-mul/s\n", v == 0 ? "8x32 product scanning (field.h)" : "9x29 redundant radix",
           ms, (double)n * iters * 2 / ms / 1e6);
  }
  return 0;
}
