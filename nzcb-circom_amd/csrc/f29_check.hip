// nzcb_debug_f29 (include/nzcb_internal.h): the 9x29-bit products of csrc/f29.h as the
// device compiles them (the generated one-asm-statement-per-column forms of csrc/f29_cols.h)
// over host-given operands, so a test can hold each against exact integers at the bounds
// the kernels rely on (the host build runs the portable loops, not the asm).
#include "../../include/nzcb_internal.h"
#include "common.h"
#include "f29.h"

namespace nzcb {
namespace {

// words in / out per item, by op
constexpr int kIn[7] = {0, 27, 54, 18, 36, 18, 36};
constexpr int kOut[7] = {0, 9, 18, 9, 18, 18, 9};

__device__ __forceinline__ F29 ld(const uint32_t* p) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = p[i];
  return r;
}
__device__ __forceinline__ void st(uint32_t* p, const F29& x) {
#pragma unroll
  for (int i = 0; i < 9; i++) p[i] = x.v[i];
}

template <int OP>
__global__ void __launch_bounds__(64) k_f29_check(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                  size_t count) {
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (t >= count) return;
  const uint32_t* a = in + t * kIn[OP];
  uint32_t* o = out + t * kOut[OP];
  if constexpr (OP == 1) {  // x w mod r, Shoup: (x, w, ws)
    st(o, mul_shoup(ld(a), ld(a + 9), ld(a + 18)));
  } else if constexpr (OP == 2) {  // two Shoup products interleaved
    F29 r1, r2;
    mul_shoup_x2(ld(a), ld(a + 9), ld(a + 18), ld(a + 27), ld(a + 36), ld(a + 45), r1, r2);
    st(o, r1);
    st(o + 9, r2);
  } else if constexpr (OP == 3) {  // a b 2^-261 mod q
    st(o, mul29<Fq29>(ld(a), ld(a + 9)));
  } else if constexpr (OP == 4) {  // (a b, c d) 2^-261 mod r, interleaved
    F29 r1, r2;
    mul29x2<Fr29>(ld(a), ld(a + 9), ld(a + 18), ld(a + 27), r1, r2);
    st(o, r1);
    st(o + 9, r2);
  } else if constexpr (OP == 5) {  // (a^2, c^2) 2^-261 mod q
    F29 r1, r2;
    sqr29x2(ld(a), ld(a + 9), r1, r2);
    st(o, r1);
    st(o + 9, r2);
  } else {  // (a b + c d) 2^-261 mod q
    st(o, mul2sum29(ld(a), ld(a + 9), ld(a + 18), ld(a + 27)));
  }
}

template <int OP>
void launch(const uint32_t* in, uint32_t* out, size_t count) {
  hipLaunchKernelGGL(k_f29_check<OP>, dim3((unsigned)((count + 63) / 64)), dim3(64), 0, nullptr, in, out, count);
}

}  // namespace
}  // namespace nzcb

using namespace nzcb;

extern "C" int nzcb_debug_f29(int device, int op, const uint32_t* in, size_t count, uint32_t* out, nzcb_err* err) {
  auto fail = [&](int code, const std::string& m) {
    if (err) {
      err->code = code;
      std::snprintf(err->msg, sizeof(err->msg), "%s", m.c_str());
    }
    return code;
  };
  if (op < 1 || op > 6 || (count && (!in || !out)) || count > (size_t(1) << 24))
    return fail(NZCB_ERR_ARG, "f29 check: op 1..6, count <= 2^24");
  try {
    if (count) {
      NZ_HIP(hipSetDevice(device));
      DevBuf<uint32_t> din(count * kIn[op]), dout(count * kOut[op]);
      NZ_HIP(hipMemcpy(din.p, in, count * kIn[op] * 4, hipMemcpyHostToDevice));
      switch (op) {
        case 1: launch<1>(din.p, dout.p, count); break;
        case 2: launch<2>(din.p, dout.p, count); break;
        case 3: launch<3>(din.p, dout.p, count); break;
        case 4: launch<4>(din.p, dout.p, count); break;
        case 5: launch<5>(din.p, dout.p, count); break;
        default: launch<6>(din.p, dout.p, count); break;
      }
      NZ_HIP(hipGetLastError());
      NZ_HIP(hipMemcpy(out, dout.p, count * kOut[op] * 4, hipMemcpyDeviceToHost));
    }
    if (err) err->code = 0;
    return 0;
  } catch (const Error& e) {
    return fail(e.code, e.what());
  } catch (const std::exception& e) {
    return fail(NZCB_ERR_INTERNAL, e.what());
  }
}
