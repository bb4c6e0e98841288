// Keccak-256 (original padding 0x01) for the Fiat-Shamir transcript.
// Replaces js-sha3@0.8.0 keccak256 used by snarkjs hashToFr
// (/root/reference/yarn.lock:5074-5077). Host-side:
// a few hundred bytes per proof.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>

namespace nzcb {

inline void keccak_f1600(uint64_t s[25]) {
  static const uint64_t RC[24] = {
      0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
      0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
      0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
      0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
      0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
      0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
  static const int ROTC[24] = {1, 3, 6, 10, 15, 21, 28, 36, 45, 55, 2, 14, 27, 41, 56, 8, 25, 43, 62, 18, 39, 61, 20, 44};
  static const int PILN[24] = {10, 7, 11, 17, 18, 3, 5, 16, 8, 21, 24, 4, 15, 23, 19, 13, 12, 2, 20, 14, 22, 9, 6, 1};
  auto rol = [](uint64_t x, int n) { return (x << n) | (x >> (64 - n)); };
  for (int r = 0; r < 24; r++) {
    uint64_t bc[5];
    for (int i = 0; i < 5; i++) bc[i] = s[i] ^ s[i + 5] ^ s[i + 10] ^ s[i + 15] ^ s[i + 20];
    for (int i = 0; i < 5; i++) {
      uint64_t t = bc[(i + 4) % 5] ^ rol(bc[(i + 1) % 5], 1);
      for (int j = 0; j < 25; j += 5) s[j + i] ^= t;
    }
    uint64_t t = s[1];
    for (int i = 0; i < 24; i++) {
      int j = PILN[i];
      uint64_t tmp = s[j];
      s[j] = rol(t, ROTC[i]);
      t = tmp;
    }
    for (int j = 0; j < 25; j += 5) {
      uint64_t b[5];
      for (int i = 0; i < 5; i++) b[i] = s[j + i];
      for (int i = 0; i < 5; i++) s[j + i] ^= (~b[(i + 1) % 5]) & b[(i + 2) % 5];
    }
    s[0] ^= RC[r];
  }
}

inline void keccak256(const uint8_t* data, size_t len, uint8_t out[32]) {
  uint64_t s[25];
  std::memset(s, 0, sizeof(s));
  const size_t rate = 136;
  uint8_t block[136];
  size_t off = 0;
  for (;;) {
    size_t take = len - off < rate ? len - off : rate;
    std::memset(block, 0, rate);
    std::memcpy(block, data + off, take);
    bool last = take < rate;
    if (last) {
      block[take] ^= 0x01;
      block[rate - 1] ^= 0x80;
    }
    for (size_t i = 0; i < rate / 8; i++) {
      uint64_t w;
      std::memcpy(&w, block + 8 * i, 8);
      s[i] ^= w;
    }
    keccak_f1600(s);
    off += take;
    if (last) break;
  }
  std::memcpy(out, s, 32);
}

}  // namespace nzcb
