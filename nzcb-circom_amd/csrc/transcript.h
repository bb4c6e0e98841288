// Fiat-Shamir transcript encodings shared by the prover and the verifier (snarkjs
// 0.4.12 plonk_prove.js / plonk_verify.js [EXT]): keccak256
// (js-sha3 0.8.0, /root/reference/yarn.lock:5074) over big-endian Fr and
// uncompressed big-endian G1 (infinity = 0x40 followed by zeros), hashToFr =
// big-endian digest mod r.
#pragma once
#include <cstring>
#include <vector>

#include "ec.h"
#include "keccak.h"

namespace nzcb {

inline Fr fr_from_le_normal(const uint8_t* p) {
  Fr x;
  std::memcpy(x.v, p, 32);
  // reduce (values from files may be >= r only if malformed; keep exact for < 2^256)
  for (int k = 0; k < 6; k++) {
    Fr y = reduce_once(x);
    if (y == x) break;
    x = y;
  }
  return to_mont(x);
}

inline void fr_to_le_normal(const Fr& m, uint8_t* out) {
  Fr x = from_mont(m);
  std::memcpy(out, x.v, 32);
}

inline void fr_to_be(const Fr& m, uint8_t* out) {
  uint8_t le[32];
  fr_to_le_normal(m, le);
  for (int i = 0; i < 32; i++) out[i] = le[31 - i];
}

inline void g1_uncompressed(const G1Affine& a, uint8_t* out) {
  if (a.is_inf()) {
    std::memset(out, 0, 64);
    out[0] = 0x40;
    return;
  }
  Fq x = from_mont(a.x), y = from_mont(a.y);
  for (int i = 0; i < 32; i++) {
    out[i] = ((const uint8_t*)x.v)[31 - i];
    out[32 + i] = ((const uint8_t*)y.v)[31 - i];
  }
}

inline Fr hash_to_fr(const std::vector<uint8_t>& data) {
  uint8_t h[32];
  keccak256(data.data(), data.size(), h);
  uint8_t le[32];
  for (int i = 0; i < 32; i++) le[i] = h[31 - i];
  return fr_from_le_normal(le);
}


}  // namespace nzcb
