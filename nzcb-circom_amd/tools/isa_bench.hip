// Instruction-throughput probe for the Montgomery-product building blocks on gfx950:
// v_mad_u64_u32, v_addc_co_u32, s_nop, v_fma_f64, v_mul_lo_u32, v_mul_hi_u32.
// Full-chip throughput (many waves) of 16 independent instructions per asm block.
#include <hip/hip_runtime.h>

#include <cstdio>

#define REP16(x) x x x x x x x x x x x x x x x x

template <int K>
__global__ void probe(uint64_t* out, int iters) {
  uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t x = threadIdx.x * 3 + 1, y = threadIdx.x * 7 + 5;
  double d0 = x, d1 = y, d2 = x + 1.0, d3 = y + 1.0, d4 = 0.5, d5 = 0.25, d6 = 0.125, d7 = 2.0;
  uint32_t h = 0;
  const uint64_t b64 = (uint64_t)threadIdx.x * 977;
  uint32_t r0 = x, r1 = x + 1, r2 = x + 2, r3 = x + 3, r4 = x + 4, r5 = x + 5, r6 = x + 6, r7 = x + 7;
  float f0 = x, f1 = y, f2 = 1.f, f3 = 2.f, f4 = 3.f, f5 = 4.f, f6 = 5.f, f7 = 6.f;
  for (int i = 0; i < iters; i++) {
    if (K == 0) {  // 16 x v_mad_u64_u32 (8 independent accumulators, 2 rounds)
      asm volatile(
          "v_mad_u64_u32 %0, vcc, %8, %9, %0\n v_mad_u64_u32 %1, vcc, %8, %9, %1\n"
          "v_mad_u64_u32 %2, vcc, %8, %9, %2\n v_mad_u64_u32 %3, vcc, %8, %9, %3\n"
          "v_mad_u64_u32 %4, vcc, %8, %9, %4\n v_mad_u64_u32 %5, vcc, %8, %9, %5\n"
          "v_mad_u64_u32 %6, vcc, %8, %9, %6\n v_mad_u64_u32 %7, vcc, %8, %9, %7\n"
          "v_mad_u64_u32 %0, vcc, %8, %9, %0\n v_mad_u64_u32 %1, vcc, %8, %9, %1\n"
          "v_mad_u64_u32 %2, vcc, %8, %9, %2\n v_mad_u64_u32 %3, vcc, %8, %9, %3\n"
          "v_mad_u64_u32 %4, vcc, %8, %9, %4\n v_mad_u64_u32 %5, vcc, %8, %9, %5\n"
          "v_mad_u64_u32 %6, vcc, %8, %9, %6\n v_mad_u64_u32 %7, vcc, %8, %9, %7\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "v"(x), "v"(y)
          : "vcc");
    } else if (K == 29) {  // 16 dependent v_mad_u64_u32 (one accumulation chain, as in mul29)
      asm volatile(REP16("v_mad_u64_u32 %0, vcc, %1, %2, %0\n") : "+v"(a0) : "v"(x), "v"(y) : "vcc");
    } else if (K == 30) {  // 2 interleaved chains
      asm volatile(REP16("v_mad_u64_u32 %0, vcc, %2, %3, %0\n v_mad_u64_u32 %1, vcc, %2, %3, %1\n")
                   : "+v"(a0), "+v"(a1) : "v"(x), "v"(y) : "vcc");
    } else if (K == 1) {  // 16 x v_add_co_u32
      asm volatile(REP16("v_add_co_u32 %0, vcc, %0, %1\n") : "+v"(x) : "v"(y) : "vcc");
    } else if (K == 2) {  // 16 x s_nop 1
      asm volatile(REP16("s_nop 1\n"));
    } else if (K == 3) {  // 16 x v_fma_f64 (8 independent)
      asm volatile(
          "v_fma_f64 %0, %0, %8, %9\n v_fma_f64 %1, %1, %8, %9\n v_fma_f64 %2, %2, %8, %9\n v_fma_f64 %3, %3, %8, %9\n"
          "v_fma_f64 %4, %4, %8, %9\n v_fma_f64 %5, %5, %8, %9\n v_fma_f64 %6, %6, %8, %9\n v_fma_f64 %7, %7, %8, %9\n"
          "v_fma_f64 %0, %0, %8, %9\n v_fma_f64 %1, %1, %8, %9\n v_fma_f64 %2, %2, %8, %9\n v_fma_f64 %3, %3, %8, %9\n"
          "v_fma_f64 %4, %4, %8, %9\n v_fma_f64 %5, %5, %8, %9\n v_fma_f64 %6, %6, %8, %9\n v_fma_f64 %7, %7, %8, %9\n"
          : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)
          : "v"(0.999), "v"(0.001));
    } else if (K == 4) {  // 16 x v_mul_lo_u32
      asm volatile(REP16("v_mul_lo_u32 %0, %0, %1\n") : "+v"(x) : "v"(y));
    } else if (K == 5) {  // 16 x v_mul_hi_u32
      asm volatile(REP16("v_mul_hi_u32 %0, %0, %1\n") : "+v"(x) : "v"(y));
    } else if (K == 7) {  // 16 x v_add_u32, 8 independent
      asm volatile(REP16("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
                         "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n")
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) : "v"(y));
    } else if (K == 8) {  // v_add_co_u32, 8 independent
      asm volatile(REP16("v_add_co_u32 %0, vcc, %0, %8\n v_add_co_u32 %1, vcc, %1, %8\n v_add_co_u32 %2, vcc, %2, %8\n"
                         "v_add_co_u32 %3, vcc, %3, %8\n v_add_co_u32 %4, vcc, %4, %8\n v_add_co_u32 %5, vcc, %5, %8\n"
                         "v_add_co_u32 %6, vcc, %6, %8\n v_add_co_u32 %7, vcc, %7, %8\n")
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) : "v"(y) : "vcc");
    } else if (K == 9) {  // v_addc_co_u32 (VOP2, vcc in/out), 8 independent
      asm volatile(REP16("v_addc_co_u32 %0, vcc, %0, %8, vcc\n v_addc_co_u32 %1, vcc, %1, %8, vcc\n"
                         "v_addc_co_u32 %2, vcc, %2, %8, vcc\n v_addc_co_u32 %3, vcc, %3, %8, vcc\n"
                         "v_addc_co_u32 %4, vcc, %4, %8, vcc\n v_addc_co_u32 %5, vcc, %5, %8, vcc\n"
                         "v_addc_co_u32 %6, vcc, %6, %8, vcc\n v_addc_co_u32 %7, vcc, %7, %8, vcc\n")
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) : "v"(y) : "vcc");
    } else if (K == 10) {  // v_add3_u32, 8 independent
      asm volatile(REP16("v_add3_u32 %0, %0, %8, %9\n v_add3_u32 %1, %1, %8, %9\n v_add3_u32 %2, %2, %8, %9\n"
                         "v_add3_u32 %3, %3, %8, %9\n v_add3_u32 %4, %4, %8, %9\n v_add3_u32 %5, %5, %8, %9\n"
                         "v_add3_u32 %6, %6, %8, %9\n v_add3_u32 %7, %7, %8, %9\n")
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) : "v"(y), "v"(x));
    } else if (K == 11) {  // v_mad_u32_u24, 8 independent
      asm volatile(REP16("v_mad_u32_u24 %0, %0, %8, %9\n v_mad_u32_u24 %1, %1, %8, %9\n v_mad_u32_u24 %2, %2, %8, %9\n"
                         "v_mad_u32_u24 %3, %3, %8, %9\n v_mad_u32_u24 %4, %4, %8, %9\n v_mad_u32_u24 %5, %5, %8, %9\n"
                         "v_mad_u32_u24 %6, %6, %8, %9\n v_mad_u32_u24 %7, %7, %8, %9\n")
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) : "v"(y), "v"(x));
    } else if (K == 12) {  // v_mul_lo_u32, 8 independent
      asm volatile(REP16("v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n"
                         "v_mul_lo_u32 %3, %3, %8\n v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n"
                         "v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8\n")
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) : "v"(y));
    } else if (K == 13) {  // v_fma_f32, 8 independent (reference: 2 cycles per wave64)
      asm volatile(REP16("v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n"
                         "v_fma_f32 %3, %3, %8, %9\n v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n"
                         "v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9\n")
                   : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7)
                   : "v"(0.999f), "v"(0.001f));
    } else if (K == 14) {  // v_mad_u64_u32 + v_addc_co_u32 pairs, 4 independent column chains
      asm volatile(REP16("v_mad_u64_u32 %0, s[20:21], %8, %9, %0\n v_mad_u64_u32 %1, s[22:23], %8, %9, %1\n"
                         "v_addc_co_u32_e64 %4, s[20:21], %4, 0, s[20:21]\n v_addc_co_u32_e64 %5, s[22:23], %5, 0, s[22:23]\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) : "v"(x), "v"(y)
                   : "s20", "s21", "s22", "s23");
    } else if (K >= 15 && K <= 28) {
#define NZ_OP8(OP) asm volatile(REP16(OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)) \
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) : "v"(y), "v"(x))
#define NZ_OP8W(OP) asm volatile(REP16(OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)) \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(y), "v"(x), "v"(b64))
#define AND(i) "v_and_b32 %" #i ", %" #i ", %8\n"
#define ALIGN(i) "v_alignbit_b32 %" #i ", %" #i ", %8, 29\n"
#define SHR(i) "v_lshrrev_b32 %" #i ", 29, %" #i "\n"
#define MU24(i) "v_mul_u32_u24 %" #i ", %" #i ", %8\n"
#define MHU24(i) "v_mul_hi_u32_u24 %" #i ", %" #i ", %8\n"
#define BFE(i) "v_bfe_u32 %" #i ", %" #i ", 3, 29\n"
#define SHR64(i) "v_lshrrev_b64 %" #i ", 29, %" #i "\n"
#define LSHLADD64(i) "v_lshl_add_u64 %" #i ", %" #i ", 0, %10\n"
#define ADD64CO(i) "v_add_co_u32 %" #i ", vcc, %" #i ", %8\n"
#define CND(i) "v_cndmask_b32 %" #i ", %" #i ", %8, vcc\n"
#define CND64(i) "v_cndmask_b32_e64 %" #i ", %" #i ", %8, s[20:21]\n"
#define BFI(i) "v_bfi_b32 %" #i ", %9, %" #i ", %8\n"
#define SUBB(i) "v_subb_co_u32 %" #i ", vcc, %" #i ", %8, vcc\n"
#define SUBCND(i) "v_subb_co_u32 %" #i ", vcc, %" #i ", %8, vcc\n v_cndmask_b32 %" #i ", %" #i ", %8, vcc\n"
      if (K == 15) NZ_OP8(AND);
      else if (K == 16) NZ_OP8(ALIGN);
      else if (K == 17) NZ_OP8(SHR);
      else if (K == 18) NZ_OP8(MU24);
      else if (K == 19) NZ_OP8(MHU24);
      else if (K == 20) NZ_OP8(BFE);
      else if (K == 21) NZ_OP8W(SHR64);
      else if (K == 22) NZ_OP8W(LSHLADD64);
      else if (K == 23) NZ_OP8(CND);
      else if (K == 24) NZ_OP8(ADD64CO);
      else if (K == 25) { asm volatile("s_mov_b64 s[20:21], -1" ::: "s20", "s21");
        asm volatile(REP16(CND64(0) CND64(1) CND64(2) CND64(3) CND64(4) CND64(5) CND64(6) CND64(7))
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) : "v"(y), "v"(x)
                   : "s20", "s21"); }
      else if (K == 26) NZ_OP8(BFI);
      else if (K == 27) { asm volatile(REP16(SUBB(0) SUBB(1) SUBB(2) SUBB(3) SUBB(4) SUBB(5) SUBB(6) SUBB(7))
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) : "v"(y), "v"(x)
                   : "vcc"); }
      else { asm volatile(REP16(SUBCND(0) SUBCND(1) SUBCND(2) SUBCND(3))
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) : "v"(y), "v"(x)
                   : "vcc"); }
    } else if (K == 6) {  // 8 x (mad; s_nop 1; addc) as in field.h mac
      asm volatile(
          "v_mad_u64_u32 %0, s[20:21], %2, %3, %0\n s_nop 1\n v_addc_co_u32_e64 %1, s[20:21], %1, 0, s[20:21]\n"
          "v_mad_u64_u32 %0, s[20:21], %2, %3, %0\n s_nop 1\n v_addc_co_u32_e64 %1, s[20:21], %1, 0, s[20:21]\n"
          "v_mad_u64_u32 %0, s[20:21], %2, %3, %0\n s_nop 1\n v_addc_co_u32_e64 %1, s[20:21], %1, 0, s[20:21]\n"
          "v_mad_u64_u32 %0, s[20:21], %2, %3, %0\n s_nop 1\n v_addc_co_u32_e64 %1, s[20:21], %1, 0, s[20:21]\n"
          "v_mad_u64_u32 %0, s[20:21], %2, %3, %0\n s_nop 1\n v_addc_co_u32_e64 %1, s[20:21], %1, 0, s[20:21]\n"
          "v_mad_u64_u32 %0, s[20:21], %2, %3, %0\n s_nop 1\n v_addc_co_u32_e64 %1, s[20:21], %1, 0, s[20:21]\n"
          "v_mad_u64_u32 %0, s[20:21], %2, %3, %0\n s_nop 1\n v_addc_co_u32_e64 %1, s[20:21], %1, 0, s[20:21]\n"
          "v_mad_u64_u32 %0, s[20:21], %2, %3, %0\n s_nop 1\n v_addc_co_u32_e64 %1, s[20:21], %1, 0, s[20:21]\n"
          : "+v"(a0), "+v"(h)
          : "v"(x), "v"(y)
          : "s20", "s21");
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ x ^ h ^
                                               (uint64_t)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7) ^
                                               (r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7) ^
                                               (uint64_t)(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7);
}

template <int K>
double run(uint64_t* d, int blocks, int threads, int iters) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  probe<K><<<blocks, threads>>>(d, 2);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  probe<K><<<blocks, threads>>>(d, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  const int blocks = 256 * 8, threads = 256, iters = 4000;
  uint64_t* d;
  (void)hipMalloc(&d, (size_t)blocks * threads * 8);
  const int NK = 29;
  const char* names[NK] = {"v_mad_u64_u32 x8", "v_add_co_u32 chain", "s_nop 1", "v_fma_f64 x8", "v_mul_lo_u32 chain",
                           "v_mul_hi_u32 chain", "mac(mad;nop;addc)", "v_add_u32 x8", "v_add_co_u32 x8",
                           "v_addc_co_u32 x8", "v_add3_u32 x8", "v_mad_u32_u24 x8", "v_mul_lo_u32 x8",
                           "v_fma_f32 x8", "mad,mad,addc,addc x2", "v_and_b32 x8", "v_alignbit_b32 x8",
                           "v_lshrrev_b32 x8", "v_mul_u32_u24 x8", "v_mul_hi_u32_u24 x8", "v_bfe_u32 x8",
                           "v_lshrrev_b64 x8", "v_lshl_add_u64 x8", "v_cndmask_b32 x8", "v_add_co_u32(e32) x8",
                           "v_cndmask_b32_e64 sgpr x8", "v_bfi_b32 x8", "v_subb_co_u32 x8", "subb+cndmask x4"};
  double ms[NK] = {run<0>(d, blocks, threads, iters), run<1>(d, blocks, threads, iters), run<2>(d, blocks, threads, iters),
                   run<3>(d, blocks, threads, iters), run<4>(d, blocks, threads, iters), run<5>(d, blocks, threads, iters),
                   run<6>(d, blocks, threads, iters), run<7>(d, blocks, threads, iters / 8),
                   run<8>(d, blocks, threads, iters / 8), run<9>(d, blocks, threads, iters / 8),
                   run<10>(d, blocks, threads, iters / 8), run<11>(d, blocks, threads, iters / 8),
                   run<12>(d, blocks, threads, iters / 8), run<13>(d, blocks, threads, iters / 8),
                   run<14>(d, blocks, threads, iters / 4),  run<15>(d, blocks, threads, iters / 8),
                   run<16>(d, blocks, threads, iters / 8), run<17>(d, blocks, threads, iters / 8),
                   run<18>(d, blocks, threads, iters / 8), run<19>(d, blocks, threads, iters / 8),
                   run<20>(d, blocks, threads, iters / 8), run<21>(d, blocks, threads, iters / 8),
                   run<22>(d, blocks, threads, iters / 8), run<23>(d, blocks, threads, iters / 8),
                   run<24>(d, blocks, threads, iters / 8), run<25>(d, blocks, threads, iters / 8),
                   run<26>(d, blocks, threads, iters / 8), run<27>(d, blocks, threads, iters / 8),
                   run<28>(d, blocks, threads, iters / 8)};
  // dependent-chain latency: mad chains at 1, 2, 4, 8 waves per SIMD (256 CUs x 4 SIMDs)
  for (int wps = 1; wps <= 8; wps *= 2) {
    const int b = 256 * wps;  // 256-thread blocks = 4 waves = one per SIMD
    const double m1 = run<29>(d, b, 256, iters), m2 = run<30>(d, b, 256, iters / 2);
    const double nw = (double)b * 256 / 64 / 1024;  // waves per SIMD
    printf("mad chain, %d wave(s)/SIMD: 1 chain %.2f, 2 chains %.2f SIMD-cycles per mad\n", wps,
           m1 * 1e-3 * 2.4e9 / (nw * iters * 16), m2 * 1e-3 * 2.4e9 / (nw * iters / 2 * 32));
  }
  const double waves = (double)blocks * threads / 64;
  for (int k = 0; k < NK; k++) {
    // wave-instructions per iteration (mac = one mad+nop+addc group)
    double per = k == 6 ? 8 : (k >= 7 && k <= 13) || k >= 15 ? 128 : k == 14 ? 64 : 16;
    int it = (k >= 7 && k <= 13) || k >= 15 ? iters / 8 : k == 14 ? iters / 4 : iters;
    double n_instr = waves * it * per;
    double simd_cycles = ms[k] * 1e-3 * 2.4e9 * 1024;    // 256 CUs x 4 SIMDs at 2.4 GHz
    printf("%-20s %8.3f ms  %6.2f SIMD-cycles per wave-instruction\n", names[k], ms[k], simd_cycles / n_instr);
  }
  return 0;
}
