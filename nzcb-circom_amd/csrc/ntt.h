// Fr radix-2 NTT / iNTT over natural-order data.
#pragma once
#include "f29.h"
#include "common.h"

namespace nzcb {

// Roots of unity, ffjavascript convention: w[28] = 5^((r-1)/2^28), w[k-1] = w[k]^2.
Fr fr_root_of_unity(int k);  // Montgomery form

struct NttTables {
  int max_log = 0;
  // Per-stage compact twiddles: stage g (butterfly span 2^g) uses w_{2^(g+1)}^k,
  // k < 2^g, stored contiguously at offset 2^g - 1, so the twiddles of consecutive
  // butterflies of a stage are consecutive in memory (coalesced 32-byte loads).
  DevBuf<Fr> fwd, inv;  // 2^max_log - 1 entries each
  // The same twiddles as split29 of their Montgomery-261 form (w * 2^261 mod r), the
  // operand of mul_fr29 (f29.h) in the butterflies
  DevBuf<F29> fwd29, inv29;
  void init(int max_log, hipStream_t st);
};

// Optional fused prologue / epilogue (coset NTTs of zero-padded polynomials):
//   input  j: in[j] * in_lo[j & 4095] * in_hi[j >> 12] for j < in_len, 0 beyond (not read)
//   output j: out[j] * out_lo[j & 4095] * out_hi[j >> 12]; sets *out_flags if an output
//             at j >= out_limit is nonzero
struct NttIo {
  size_t in_len = ~size_t(0);
  const Fr* in_lo = nullptr;
  const Fr* in_hi = nullptr;
  const Fr* out_lo = nullptr;
  const Fr* out_hi = nullptr;
  size_t out_limit = ~size_t(0);
  uint32_t* out_flags = nullptr;
};

// out = NTT(in) (inverse: out = (1/N) * iNTT(in)), N = 2^log_n <= 2^max_log.
// Natural order in and out; in != out required (first pass gathers in bit-reversed order).
// scale (optional, Montgomery) multiplies every input element on load.
void ntt(const NttTables& t, const Fr* in, Fr* out, int log_n, bool inverse, hipStream_t st,
         const Fr* scale = nullptr, const NttIo* io = nullptr);

}  // namespace nzcb
