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
  // butterflies of a stage are consecutive in memory (coalesced loads); 2^max_log - 1
  // entries each, as the operand pair of f29.h's Shoup product: the twiddle's value w
  // (canonical, not Montgomery: x in Montgomery-256 times w stays Montgomery-256) and
  // ws = floor(w 2^261 / r)
  struct Tw {
    F29 w, ws;
  };
  DevBuf<Tw> fwd29, inv29;
  // Inter-pass scratch of the 9x29 pipeline (ntt29_pass_kernel): limb-major [9][2^max_log]
  // u32, the transform's values between its HBM passes (one transform at a time: every
  // caller runs its NTTs on one stream)
  DevBuf<uint32_t> scratch29;
  void init(int max_log, hipStream_t st);
};

// Optional fused prologue / epilogue (coset NTTs of zero-padded polynomials). Factors
// are split29 of their Montgomery-261 form (f * 2^261 mod r, as the twiddles), one
// 9x29 product per element:
//   input  j: in[j] * in_f[j] for j < in_len, 0 beyond (not read)
//   output j: out[j] * out_f[j]; sets *out_flags if an output at j >= out_limit is
//             nonzero. out_f_has_scale: out_f already holds the inverse transform's
//             1/N (the first pass then skips it).
//   fold (a polynomial of degree < n + fold_len evaluated where x^n = d): input j <
//             fold_len also adds in[j + fold_n] * d, before in_f (fold_f: d's operand)
struct NttIo {
  size_t in_len = ~size_t(0);
  const F29* in_f = nullptr;
  size_t fold_len = 0, fold_n = 0;
  F29 fold_f = {};
  const F29* out_f = nullptr;
  bool out_f_has_scale = false;
  size_t out_limit = ~size_t(0);
  uint32_t* out_flags = nullptr;
};

// out = NTT(in) (inverse: out = (1/N) * iNTT(in)), N = 2^log_n <= 2^max_log.
// Natural order in and out; in != out required (first pass gathers in bit-reversed order).
// scale (optional, Montgomery) multiplies every input element on load.
// scratch29 (optional): 9 << log_n words for the inter-pass values instead of t.scratch29,
// so that transforms on two streams can run at once (the prover's round 2).
void ntt(const NttTables& t, const Fr* in, Fr* out, int log_n, bool inverse, hipStream_t st,
         const Fr* scale = nullptr, const NttIo* io = nullptr, uint32_t* scratch29 = nullptr);

}  // namespace nzcb
