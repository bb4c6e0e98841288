// Witness VM: runs a circuit's witness program (nzcb/circuit.py Circuit.write_program)
// on the GPU, one workgroup per witness, in place of the circom wasm witness calculator
// (circom_runtime 0.1.17, /root/reference/yarn.lock:2496; called by snarkjs
// plonk.fullProve's wtns_calculate). For nzcp_live the program
// is NZCPPubIdentity(1, 351, 0, 4, 2, 4) (nzcb/nzcpgen.py).
//
// Program format (little endian):
//   "nzwp" u32 version n_wires n_out n_pub_in n_prv_in n_consts n_terms n_ops n_levels
//   consts[n_consts] 32 B normal form | terms[n_terms] (u32 wire, u32 const) |
//   ops[n_ops] 8 x u32 {type | err << 8 | n << 16, dst, a_off, a_n, b_off, b_n, c_off, c_n}
//   level_start[n_levels + 1] u32 | level_macro_start[n_levels] u32 |
//   u32 n_names, then per main input: u32 len, name bytes, u32 size (declaration order)
//   [optional, nzcb_wprog_remap] "wmap" u32 T, T x u32: output wire t = program wire
//   map[t], so the witness comes out in another wire order (e.g. circom's, by signal
//   name from two .sym files); the program runs into scratch and a gather reorders
// Ops are sorted by dependency level; inside a level the scalar ops (LIN MUL INV BITS
// CHECK) come first and are spread over the workgroup's threads, the macro ops (QUIN,
// SHA256, SHA512) follow and each runs on the whole workgroup. One barrier per level.
//
// Witness values live in HBM in normal form (what nzcb_prove_device reads). A linear
// combination is evaluated in Montgomery form with coefficients pre-scaled by R^2:
// mont_mul(w, c R^2) = (w c) R, so one product per term and one conversion per result.
// Almost every value of this circuit is a bit, a byte or a small position, and the
// heavy gadgets are macro ops that write their signals straight from integer state:
//   QUIN   QuinSelector's 2n + m signals; IsZero inverses of the small integers i - index
//          from a table of 1/1..1/kInvTable (Fermat only for a non-small index)
//   SHA*   one compression computed by lane 0 in 32/64-bit integers, then every signal
//          of the block (all in {0, 1, -1}) written by the workgroup
// A failing BITS/CHECK does an atomicMin of (creation order << 8 | err) on the pass's
// status word, so the host sees the first failure in template order, as circom throws.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace nzcb {
namespace wvm {

constexpr uint32_t kInvTable = 4096;
constexpr uint32_t kNoWire = 0xFFFFFFFFu;
constexpr uint32_t kWaveTerms = 16;
// NZCB_WVM_LEVEL_CLOCK record per level: [0] after the barrier, [1 + w] wave w done with the
// thread segment, [17 + w] done with the wave segment (pass 0; development aid)
constexpr int kClockSlots = 37;  // + [33..36] SHA phases (message/state read, words, compression, signals)
enum { OP_LIN = 0, OP_MUL, OP_INV, OP_BITS, OP_CHECK, OP_QUIN, OP_SHA256, OP_SHA512 };

struct Op {
  uint32_t code, dst, a_off, a_n, b_off, b_n, c_off, c_n;
};
struct Term {  // program file
  uint32_t wire, ci;
};
struct DTerm {  // device: sc = the coefficient as a small signed integer, or kBigCoef
  uint32_t wire, ci;
  int32_t sc;
  uint32_t pad;
};
constexpr int32_t kBigCoef = INT32_MIN;

// a level's ops, reordered by the loader: [s, w) one per thread, [w, m) one per wave
// (QUIN and scalar ops with more than kWaveTerms terms), [m, e) one per workgroup (SHA)
struct Level {
  uint32_t s, w, m, e;
};

struct Prog {
  const Fr* consts;   // coefficient * R^2 mod r
  const DTerm* terms;
  const Op* ops;
  const Level* levels;
  const Fr* inv_small;  // 1/i (normal form), i < kInvTable
  uint32_t n_levels, n_wires, n_inputs, in_base;
};

// ---- SHA-2 block layout (nzcb/circuit.py sha_block_layout) --------------------------
template <int B>
struct Sha;
template <>
struct Sha<32> {
  static constexpr int R = 64, S0a = 2, S0b = 13, S0c = 22, S1a = 6, S1b = 11, S1c = 25;
  static constexpr int s0a = 7, s0b = 18, s0c = 3, s1a = 17, s1b = 19, s1c = 10;
};
template <>
struct Sha<64> {
  static constexpr int R = 80, S0a = 28, S0b = 34, S0c = 39, S1a = 14, S1b = 18, S1c = 41;
  static constexpr int s0a = 1, s0b = 8, s0c = 7, s1a = 19, s1b = 61, s1c = 6;
};

__constant__ uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
__constant__ uint32_t kSha256IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                      0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
__constant__ uint64_t kSha512K[80] = {
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
    0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
    0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
    0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
    0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
    0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
    0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
    0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
    0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
    0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
    0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
    0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
    0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
    0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
    0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
    0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
    0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};
__constant__ uint64_t kSha512IV[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                                      0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                                      0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};

template <int B>
struct ShaLayout {
  static constexpr int nx0 = 2 * B - Sha<B>::s0c;  // XOR3 signals (2 each) + XOR2 (1 each)
  static constexpr int nx1 = 2 * B - Sha<B>::s1c;
  static constexpr int sched = nx0 + nx1 + B + 2;
  static constexpr int round = 9 * B + 6;
  static constexpr int n_sched = Sha<B>::R - 16;
  static constexpr int round_base = n_sched * sched;
  static constexpr int final_base = round_base + Sha<B>::R * round;
  static constexpr int size = final_base + 8 * (B + 1);
};

// per-block integer state in LDS (lane 0 fills it, the workgroup reads it)
struct ShaShared {
  uint64_t W[80];
  uint64_t A[84], E[84];   // A[t + 4] = a after round t; A[0..3] = d, c, b, a of the input state
  uint64_t H[8];
  uint8_t wc[80], ac[80], ec[80], hc[8];  // carries of the W, new-a, new-e and final sums
  uint8_t msg[64];
  uint32_t state_bits[8 * 64 / 32];
};

__device__ __forceinline__ Fr fr_small(int v) {  // v in {0, 1, -1}
  Fr r = Fr::zero();
  if (v > 0) {
    r.v[0] = 1;
  } else if (v < 0) {
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = FrParams::P[i];
    r.v[0] -= 1;
  }
  return r;
}

__device__ __forceinline__ int bit_of(uint64_t x, int i) { return (int)((x >> i) & 1u); }

__device__ __forceinline__ void put(Fr* p, int v) {  // v in {0, 1, -1}
  *p = fr_small(v);
}

// The signals of bit i of ROTR r1 ^ ROTR r2 ^ (SHR|ROTR) r3 of word x, from o = 0 of its
// block: a XOR3 bit (i + r3 inside the word) is the pair (b & c, a ? (b == c ? 1 : -1) : 0)
// at 2i, 2i + 1; past the shift (SHR, i >= B - r3) a XOR2 bit is the single a & b at
// 2 (B - r3) + (i - (B - r3)).
template <int B>
__device__ __forceinline__ void put_xor(Fr* row, uint64_t x, int r1, int r2, int r3, bool shr, int i) {
  const int n3 = shr ? B - r3 : B;
  const int a = bit_of(x, (i + r1) % B), b = bit_of(x, (i + r2) % B);
  if (i < n3) {
    const int c = bit_of(x, shr ? i + r3 : (i + r3) % B);
    put(row + 2 * i, b & c);
    put(row + 2 * i + 1, a ? (b == c ? 1 : -1) : 0);
  } else {
    put(row + 2 * n3 + (i - n3), a & b);
  }
}

template <int B>
__device__ __forceinline__ uint64_t rotr(uint64_t x, int n) {
  if (B == 32) {
    const uint32_t y = (uint32_t)x;
    return (uint32_t)((y >> n) | (y << (32 - n)));
  }
  return (x >> n) | (x << (64 - n));
}

template <int B>
__device__ __forceinline__ uint64_t sig(uint64_t x, int r1, int r2, int r3, bool shr) {
  return rotr<B>(x, r1) ^ rotr<B>(x, r2) ^ (shr ? (x >> r3) : rotr<B>(x, r3));
}

// sum of words with carry out (k words < 8, each < 2^B)
template <int B>
__device__ __forceinline__ uint64_t addw(uint64_t acc, uint64_t x, uint32_t& carry) {
  if (B == 32) {
    const uint64_t s = acc + x;
    carry += (uint32_t)(s >> 32);
    return s & 0xffffffffull;
  }
  const uint64_t s = acc + x;
  carry += s < x;
  return s;
}

// One SHA-2 block gadget: the workgroup reads the message bits and the input state, lane 0
// runs the compression with the working variables in registers (writing each round's words
// and carries to LDS, never reading them back), then every signal of the block is written
// bit-sliced: one work item per (row, bit) writes all of that bit's signals, so no item
// branches on its position inside a row.
template <int B>
__device__ void sha_block(Fr* W, const Op& op, ShaShared& sh, uint64_t* clk) {
  using L = ShaLayout<B>;
  using S = Sha<B>;
  const int tid = threadIdx.x, nt = blockDim.x;
  const uint64_t mask = B == 64 ? ~0ull : 0xffffffffull;
  // message bytes from the byte-wise bit wires (LSB first); a wire that is not a bit
  // (only in a witness that already failed a check) contributes its lowest bit
  for (int k = tid; k < 64; k += nt) {
    uint32_t byte = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) byte |= (W[op.b_off + 8 * k + j].v[0] & 1u) << j;
    sh.msg[k] = (uint8_t)byte;
  }
  // input state: the previous block's final sums (bits LSB first + 1 carry per word)
  if (op.a_off != kNoWire) {
    for (int k = tid; k < 8 * B; k += nt) {
      const int j = k / B, i = k % B;
      const uint32_t bit = W[op.a_off + L::final_base + j * (B + 1) + i].v[0] & 1u;
      if (bit) atomicOr(&sh.state_bits[k >> 5], 1u << (k & 31));
    }
  }
  __syncthreads();
  if (clk && tid == 0) clk[33] = wall_clock64();
  if (tid < 16) {  // message words (big endian)
    const int nbw = B / 8;
    uint64_t x = 0;
    if (B == 32 || tid < 8) {
      for (int q = 0; q < nbw; q++) x = (x << 8) | sh.msg[nbw * tid + q];
    } else {  // SHA-512 of a 64-byte message: 0x80, zeros, 128-bit length 512
      x = tid == 8 ? 1ull << 63 : (tid == 15 ? 512 : 0);
    }
    sh.W[tid] = x;
  } else if (tid >= 64 && tid < 72) {  // input state words
    const int j = tid - 64;
    uint64_t x = 0;
    if (op.a_off == kNoWire) {
      x = B == 32 ? (uint64_t)kSha256IV[j] : kSha512IV[j];
    } else {
      for (int i = 0; i < B; i++) {
        const int k = j * B + i;
        x |= (uint64_t)((sh.state_bits[k >> 5] >> (k & 31)) & 1u) << i;
      }
    }
    sh.H[j] = x;
  }
  __syncthreads();
  if (clk && tid == 0) clk[34] = wall_clock64();
  if (tid == 0) {
    uint64_t H[8];
#pragma unroll
    for (int j = 0; j < 8; j++) H[j] = sh.H[j];
    // A[0..3] = d, c, b, a; E[0..3] = h, g, f, e
    sh.A[3] = H[0]; sh.A[2] = H[1]; sh.A[1] = H[2]; sh.A[0] = H[3];
    sh.E[3] = H[4]; sh.E[2] = H[5]; sh.E[1] = H[6]; sh.E[0] = H[7];
    uint64_t a = H[0], b = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
    for (int t = 0; t < S::R; t++) {
      uint64_t wt;
      if (t < 16) {
        wt = sh.W[t];
      } else {
        uint32_t cw = 0;
        wt = sig<B>(sh.W[t - 2], S::s1a, S::s1b, S::s1c, true);
        wt = addw<B>(wt, sh.W[t - 7], cw);
        wt = addw<B>(wt, sig<B>(sh.W[t - 15], S::s0a, S::s0b, S::s0c, true), cw);
        wt = addw<B>(wt, sh.W[t - 16], cw);
        sh.W[t] = wt;
        sh.wc[t] = (uint8_t)cw;
      }
      const uint64_t S1 = sig<B>(e, S::S1a, S::S1b, S::S1c, false);
      const uint64_t ch = (e & f) ^ (~e & g & mask);
      const uint64_t S0 = sig<B>(a, S::S0a, S::S0b, S::S0c, false);
      const uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
      const uint64_t k = B == 32 ? (uint64_t)kSha256K[t] : kSha512K[t];
      uint32_t c1 = 0;  // T1 = h + S1 + ch + K + W
      uint64_t t1 = addw<B>(h, S1, c1);
      t1 = addw<B>(t1, ch, c1);
      t1 = addw<B>(t1, k, c1);
      t1 = addw<B>(t1, wt, c1);
      uint32_t ca = c1;
      uint64_t na = addw<B>(t1, S0, ca);
      na = addw<B>(na, mj, ca);
      uint32_t ce = c1;
      const uint64_t ne = addw<B>(t1, d, ce);
      sh.A[t + 4] = na;
      sh.E[t + 4] = ne;
      sh.ac[t] = (uint8_t)ca;
      sh.ec[t] = (uint8_t)ce;
      h = g; g = f; f = e; e = ne;
      d = c; c = b; b = a; a = na;
    }
    const uint64_t V[8] = {a, b, c, d, e, f, g, h};
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint32_t cf = 0;
      sh.H[j] = addw<B>(H[j], V[j], cf);  // final sums (the input state is no longer needed)
      sh.hc[j] = (uint8_t)cf;
    }
  }
  __syncthreads();
  if (clk && tid == 0) clk[35] = wall_clock64();
  Fr* out = W + op.dst;
  // message schedule rows t = 16 .. R-1: sigma0(W[t-15]) signals, sigma1(W[t-2]), W[t] bits + 2 carries
  for (int it = tid; it < L::n_sched * B; it += nt) {
    const int t = 16 + it / B, i = it % B;
    Fr* row = out + (t - 16) * L::sched;
    put_xor<B>(row, sh.W[t - 15], S::s0a, S::s0b, S::s0c, true, i);
    put_xor<B>(row + L::nx0, sh.W[t - 2], S::s1a, S::s1b, S::s1c, true, i);
    Fr* wb = row + L::nx0 + L::nx1;
    put(wb + i, bit_of(sh.W[t], i));
    if (i < 2) put(wb + B + i, (sh.wc[t] >> i) & 1);
  }
  // rounds: Sigma1(e) pairs, Ch, Sigma0(a) pairs, Maj pairs, new a bits + 3 carries, new e bits + 3 carries
  for (int it = tid; it < S::R * B; it += nt) {
    const int t = it / B, i = it % B;
    Fr* row = out + L::round_base + t * L::round;
    const uint64_t a = sh.A[t + 3], b = sh.A[t + 2], c = sh.A[t + 1];
    const uint64_t e = sh.E[t + 3], f = sh.E[t + 2], g = sh.E[t + 1];
    put_xor<B>(row, e, S::S1a, S::S1b, S::S1c, false, i);
    put(row + 2 * B + i, bit_of(e, i) ? bit_of(f, i) - bit_of(g, i) : 0);
    put_xor<B>(row + 3 * B, a, S::S0a, S::S0b, S::S0c, false, i);
    put(row + 5 * B + 2 * i, bit_of(b, i) & bit_of(c, i));
    put(row + 5 * B + 2 * i + 1, bit_of(a, i) & (bit_of(b, i) ^ bit_of(c, i)));
    put(row + 7 * B + i, bit_of(sh.A[t + 4], i));
    put(row + 8 * B + 3 + i, bit_of(sh.E[t + 4], i));
    if (i < 3) {
      put(row + 8 * B + i, (sh.ac[t] >> i) & 1);
      put(row + 9 * B + 3 + i, (sh.ec[t] >> i) & 1);
    }
  }
  // final sums: 8 words of B bits + 1 carry
  for (int it = tid; it < 8 * (B + 1); it += nt) {
    const int j = it / (B + 1), i = it % (B + 1);
    put(out + L::final_base + it, i < B ? bit_of(sh.H[j], i) : (int)(sh.hc[j] & 1u));
  }
  __syncthreads();
  if (clk && tid == 0) clk[36] = wall_clock64();
  for (int k = tid; k < 8 * 64 / 32; k += nt) sh.state_bits[k] = 0;
  __syncthreads();
}

// A linear combination is summed in two parts: terms whose coefficient is a small signed
// integer (|c| < 2^31, DTerm.sc) and whose wire value is below 2^32 go into an exact
// 128-bit integer; any other term is a Montgomery product w (c R^2) = w c R into a field
// accumulator. In nzcp_live 99% of the terms are of the first kind (bits, bytes and
// positions with coefficients +-1, +-2^k), so an op rarely multiplies in the field at all:
// a level's latency is then its loads, not a chain of 8 x 32-bit Montgomery products.
struct LcAcc {
  __int128 i;
  Fr m;
  bool slow;
};

__device__ __forceinline__ LcAcc lc_zero() {
  LcAcc a;
  a.i = 0;
  a.m = Fr::zero();
  a.slow = false;
  return a;
}

__device__ __forceinline__ bool below_2p32(const Fr& w) {
  uint32_t hi = 0;
#pragma unroll
  for (int k = 1; k < 8; k++) hi |= w.v[k];
  return hi == 0;
}

// x mod r for |x| < 2^127
__device__ __forceinline__ Fr i128_to_fr(__int128 x) {
  const bool ng = x < 0;
  const unsigned __int128 m = ng ? (unsigned __int128)(-x) : (unsigned __int128)x;
  Fr f = Fr::zero();
  f.v[0] = (uint32_t)m;
  f.v[1] = (uint32_t)(m >> 32);
  f.v[2] = (uint32_t)(m >> 64);
  f.v[3] = (uint32_t)(m >> 96);
  return ng ? neg(f) : f;
}

__device__ __forceinline__ Fr lc_value(const LcAcc& a) {
  Fr r = i128_to_fr(a.i);
  if (a.slow) r = r + from_mont(a.m);
  return r;
}

// the combination as an int64 when it is one (no field part, in range)
__device__ __forceinline__ bool lc_int64(const LcAcc& a, int64_t& v) {
  if (a.slow || a.i < (__int128)INT64_MIN || a.i > (__int128)INT64_MAX) return false;
  v = (int64_t)a.i;
  return true;
}

__device__ __forceinline__ bool lc_is_zero(const LcAcc& a) {
  return a.slow ? lc_value(a).is_zero() : a.i == 0;
}

// Term lists a | b | c (counts na, nb, nc) of an op, loading four terms, then their wires,
// at a time: a level's latency is its longest chain of dependent loads.
__device__ __forceinline__ void lcs_gather(const Prog& P, const Fr* W, const Op& op, uint32_t na, uint32_t nb,
                                           uint32_t nc, LcAcc& a, LcAcc& b, LcAcc& c) {
  a = lc_zero();
  b = lc_zero();
  c = lc_zero();
  const uint32_t nab = na + nb, tot = nab + nc;
  for (uint32_t j0 = 0; j0 < tot; j0 += 4) {
    DTerm t[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t j = j0 + q;
      if (j < tot) t[q] = P.terms[j < na ? op.a_off + j : (j < nab ? op.b_off + (j - na) : op.c_off + (j - nab))];
    }
    Fr w[4];
#pragma unroll
    for (int q = 0; q < 4; q++)
      if (j0 + q < tot) w[q] = W[t[q].wire];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t j = j0 + q;
      if (j < tot) {
        int64_t p = 0;
        Fr x = Fr::zero();
        const bool fast = t[q].sc != kBigCoef && below_2p32(w[q]);
        if (fast)
          p = (int64_t)t[q].sc * (int64_t)w[q].v[0];
        else
          x = w[q] * P.consts[t[q].ci];
        const int seg = j < na ? 0 : (j < nab ? 1 : 2);  // selects, not a reference (scratch)
        a.i += seg == 0 ? p : 0;
        b.i += seg == 1 ? p : 0;
        c.i += seg == 2 ? p : 0;
        if (!fast) {
          if (seg == 0) {
            a.m = a.m + x;
            a.slow = true;
          } else if (seg == 1) {
            b.m = b.m + x;
            b.slow = true;
          } else {
            c.m = c.m + x;
            c.slow = true;
          }
        }
      }
    }
  }
}

// one linear combination over a whole wave: lane i sums terms i, i + 64, ..., then a
// butterfly of shuffles leaves the total (a sum mod r, so order-free) in every lane
__device__ __forceinline__ Fr lc_wave(const Prog& P, const Fr* W, uint32_t off, uint32_t n, int lane) {
  LcAcc acc = lc_zero();
  for (uint32_t i = lane; i < n; i += 64) {
    const DTerm t = P.terms[off + i];
    const Fr w = W[t.wire];
    if (t.sc != kBigCoef && below_2p32(w)) {
      acc.i += (int64_t)t.sc * (int64_t)w.v[0];
    } else {
      acc.m = acc.m + w * P.consts[t.ci];
      acc.slow = true;
    }
  }
  Fr v = lc_value(acc);
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    Fr o;
#pragma unroll
    for (int k = 0; k < 8; k++) o.v[k] = (uint32_t)__shfl_xor((int)v.v[k], d, 64);
    v = v + o;
  }
  return v;
}

// limb k of x without indexing a register array by a variable (that would go to scratch)
__device__ __forceinline__ uint32_t limb(const Fr& x, uint32_t k) {
  uint32_t r = x.v[0];
#pragma unroll
  for (int q = 1; q < 8; q++) r = k == (uint32_t)q ? x.v[q] : r;
  return r;
}

// normal-form x as a small signed integer: 1 = non-negative (val), -1 = negative (r - val), 0 = large
__device__ __forceinline__ int small_int(const Fr& x, uint32_t& val) {
  uint32_t hi = 0;
#pragma unroll
  for (int i = 1; i < 8; i++) hi |= x.v[i];
  if (hi == 0 && x.v[0] < 0x40000000u) {
    val = x.v[0];
    return 1;
  }
  const Fr nx = neg(x);
  hi = 0;
#pragma unroll
  for (int i = 1; i < 8; i++) hi |= nx.v[i];
  if (hi == 0 && nx.v[0] < 0x40000000u) {
    val = nx.v[0];
    return -1;
  }
  return 0;
}

__device__ Fr inv_normal(const Prog& P, const Fr& x) {
  uint32_t m;
  const int s = small_int(x, m);
  if (s != 0 && m < kInvTable) {
    if (m == 0) return Fr::zero();
    const Fr r = P.inv_small[m];
    return s > 0 ? r : neg(r);
  }
  return from_mont(inverse(to_mont(x)));
}

__device__ __forceinline__ void fail(uint32_t* status, uint32_t order, uint32_t err) {
  atomicMin(status, (order << 8) | err);
}

// term lists a scalar op evaluates: LIN/INV/BITS a; CHECK a, b; MUL a, b, c
__device__ __host__ __forceinline__ void op_counts(const Op& op, uint32_t& na, uint32_t& nb, uint32_t& nc) {
  const uint32_t typ = op.code & 0xFF;
  na = op.a_n;
  nb = (typ == OP_MUL || typ == OP_CHECK) ? op.b_n : 0;
  nc = typ == OP_MUL ? op.c_n : 0;
}

// a scalar op from its linear combinations; lane / stride split the stores (1 thread:
// 0 / 1; a wave: every lane holds the same values, lane 0 stores, BITS spread over lanes)
template <class V>
__device__ void finish_op(const Prog& P, Fr* W, const Op& op, V va, V vb, V vc, uint32_t* status, uint32_t lane,
                          uint32_t stride) {
  const uint32_t typ = op.code & 0xFF, err = (op.code >> 8) & 0xFF, n = op.code >> 16;
  switch (typ) {
    case OP_LIN: {
      const Fr r = va();
      if (lane == 0) W[op.dst] = r;
      break;
    }
    case OP_MUL: {
      const Fr r = va.mul_add(vb, vc);
      if (lane == 0) W[op.dst] = r;
      break;
    }
    case OP_INV: {
      const Fr r = inv_normal(P, va());
      if (lane == 0) W[op.dst] = r;
      break;
    }
    case OP_BITS: {
      const Fr x = va();
      for (uint32_t i = lane; i < n; i += stride) {
        Fr bit = Fr::zero();
        bit.v[0] = (limb(x, i >> 5) >> (i & 31)) & 1u;
        W[op.dst + i] = bit;
      }
      uint32_t big = 0;  // any bit >= n set
#pragma unroll
      for (uint32_t k = 0; k < 8; k++) {
        const uint32_t lo = 32 * k;
        const uint32_t keep = n <= lo ? ~0u : (n >= lo + 32 ? 0u : ~0u << (n - lo));
        big |= x.v[k] & keep;
      }
      if (big && lane == 0) fail(status, op.c_off, err);
      break;
    }
    case OP_CHECK: {
      // a (x b when b is present) == 0; a field has no zero divisors
      const bool zero = va.is_zero() || (op.b_n && vb.is_zero());
      if (!zero && lane == 0) fail(status, op.c_off, err);
      break;
    }
    default:
      if (lane == 0) fail(status, 0xFFFFFFu, 0xFE);
  }
}

// an op's combination as summed by one thread (exact integer + field part)
struct LcVal {
  const LcAcc& a;
  __device__ Fr operator()() const { return lc_value(a); }
  __device__ bool is_zero() const { return lc_is_zero(a); }
  __device__ Fr mul_add(const LcVal& b, const LcVal& c) const {
    int64_t x, y, z;
    if (lc_int64(a, x) && lc_int64(b.a, y) && lc_int64(c.a, z)) return i128_to_fr((__int128)x * y + z);
    return to_mont(lc_value(a)) * lc_value(b.a) + lc_value(c.a);  // (a R) b / R = a b
  }
};

// an op's combination as a field element (wave reductions)
struct FrVal {
  Fr x;
  __device__ Fr operator()() const { return x; }
  __device__ bool is_zero() const { return x.is_zero(); }
  __device__ Fr mul_add(const FrVal& b, const FrVal& c) const { return to_mont(x) * b.x + c.x; }
};

__device__ __forceinline__ void scalar_op(const Prog& P, Fr* W, const Op& op, uint32_t* status) {
  uint32_t na, nb, nc;
  op_counts(op, na, nb, nc);
  LcAcc a, b, c;
  lcs_gather(P, W, op, na, nb, nc, a, b, c);
  finish_op(P, W, op, LcVal{a}, LcVal{b}, LcVal{c}, status, 0, 1);
}

// QuinSelector on one wave: every lane evaluates the index (same loads, so no exchange),
// then the lanes write the 2n + m signals
__device__ void quin_wave(const Prog& P, Fr* W, const Op& op, int lane) {
  const uint32_t n = op.code >> 16, m = op.b_n;
  LcAcc a, b, c;
  lcs_gather(P, W, op, op.a_n, 0, 0, a, b, c);
  const Fr fidx = lc_value(a);
  uint32_t mag = 0;
  const int sign = small_int(fidx, mag);
  const bool hit = sign > 0 && mag < m;
  const Fr sel = hit ? W[op.b_off + mag] : Fr::zero();
  const int64_t idx = sign > 0 ? (int64_t)mag : -(int64_t)mag;
  const Fr one = fr_small(1);
  for (uint32_t i = lane; i < n; i += 64) {
    Fr eq = Fr::zero(), inv;
    if (sign != 0) {
      const int64_t d = (int64_t)i - idx;
      if (d == 0) {
        eq = one;
        inv = Fr::zero();
      } else {
        const uint64_t ad = d < 0 ? (uint64_t)(-d) : (uint64_t)d;
        if (ad < kInvTable) {
          inv = d < 0 ? neg(P.inv_small[ad]) : P.inv_small[ad];
        } else {
          Fr df = Fr::zero();
          df.v[0] = (uint32_t)ad;
          df.v[1] = (uint32_t)(ad >> 32);
          inv = from_mont(inverse(to_mont(df)));
          if (d < 0) inv = neg(inv);
        }
      }
    } else {
      Fr fi = Fr::zero();
      fi.v[0] = i;
      inv = from_mont(inverse(to_mont(fi - fidx)));
    }
    W[op.dst + i] = eq;
    W[op.dst + n + i] = inv;
  }
  for (uint32_t i = lane; i < m; i += 64) W[op.dst + 2 * n + i] = (hit && i >= mag) ? sel : Fr::zero();
}

// an op of a level's wave segment: a QuinSelector or a scalar op with a long linear combination
__device__ __forceinline__ void wave_op(const Prog& P, Fr* W, const Op& op, uint32_t* status, int lane) {
  if ((op.code & 0xFF) == OP_QUIN) {
    quin_wave(P, W, op, lane);
    return;
  }
  uint32_t na, nb, nc;
  op_counts(op, na, nb, nc);
  const Fr a = lc_wave(P, W, op.a_off, na, lane);
  const Fr b = nb ? lc_wave(P, W, op.b_off, nb, lane) : Fr::zero();
  const Fr c = nc ? lc_wave(P, W, op.c_off, nc, lane) : Fr::zero();
  finish_op(P, W, op, FrVal{a}, FrVal{b}, FrVal{c}, status, lane, 64);
}

// One workgroup per pass; per level: the thread segment spread over threads, the wave
// segment over waves, the workgroup segment (SHA blocks) one op at a time, one barrier.
// Ops of one level are independent, so the three segments need no barrier between them.
// 512 threads per pass (the size the level segments are cut for; the 256 / 1024 variants
// were A/B switches without tests and were removed in round 5).
static constexpr int kWvmThreads = 512;
template <int NT>
__global__ void __launch_bounds__(NT) wvm_kernel(Prog P, const Fr* __restrict__ inputs, Fr* witness,
                                                 size_t stride_elems, uint32_t* status,
                                                 uint64_t* __restrict__ level_clock) {
  __shared__ ShaShared sh;
  constexpr int NW = NT / 64;
  const uint32_t pass = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  Fr* W = witness + (size_t)pass * stride_elems;
  const Fr* in = inputs + (size_t)pass * P.n_inputs;
  uint32_t* st = status + pass;
  if (threadIdx.x == 0) {
    *st = 0xFFFFFFFFu;
    W[0] = fr_small(1);
  }
  for (int k = threadIdx.x; k < 8 * 64 / 32; k += blockDim.x) sh.state_bits[k] = 0;
  // inputs reduced mod r (a 256-bit value is below 6r), as circom reads signals
  for (uint32_t i = threadIdx.x; i < P.n_inputs; i += blockDim.x) {
    Fr x = in[i];
#pragma unroll 1
    for (int k = 0; k < 6; k++) x = reduce_once(x);
    W[P.in_base + i] = x;
  }
  Level nxt = P.n_levels ? P.levels[0] : Level{0, 0, 0, 0};
  __syncthreads();
  if (level_clock && pass == 0 && threadIdx.x == 0) level_clock[0] = wall_clock64();
  for (uint32_t lv = 0; lv < P.n_levels; lv++) {
    const Level L = nxt;
    if (lv + 1 < P.n_levels) nxt = P.levels[lv + 1];  // static table: fetched a level ahead
    const bool clk = level_clock && pass == 0 && lane == 0;
    for (uint32_t k = L.s + threadIdx.x; k < L.w; k += NT) scalar_op(P, W, P.ops[k], st);
    if (clk) level_clock[(size_t)(lv + 1) * kClockSlots + 1 + wave] = wall_clock64();
    for (uint32_t k = L.w + wave; k < L.m; k += NW) wave_op(P, W, P.ops[k], st, lane);
    if (clk) level_clock[(size_t)(lv + 1) * kClockSlots + 17 + wave] = wall_clock64();
    for (uint32_t k = L.m; k < L.e; k++) {
      const Op op = P.ops[k];
      if ((op.code & 0xFF) == OP_SHA256)
        sha_block<32>(W, op, sh, level_clock && pass == 0 ? level_clock + (size_t)(lv + 1) * kClockSlots : nullptr);
      else
        sha_block<64>(W, op, sh, level_clock && pass == 0 ? level_clock + (size_t)(lv + 1) * kClockSlots : nullptr);
    }
    __syncthreads();
    if (level_clock && pass == 0 && threadIdx.x == 0) level_clock[(size_t)(lv + 1) * kClockSlots] = wall_clock64();
  }
}

// per-run buffers: concurrent runs of one program (the N-API addon's fullProve promises,
// each on its own thread) take a slot each, so they overlap on the GPU instead of taking
// turns; a slot's stream runs the launch when the caller passes none
struct RunSlot {
  DevBuf<uint32_t> status;
  size_t status_cap = 0;
  DevBuf<Fr> scratch;  // remapped programs: the program's own wire order
  size_t scratch_cap = 0;
  hipStream_t st = nullptr;
  hipEvent_t after_null = nullptr;  // orders the slot's stream after the null stream's work
  ~RunSlot() {
    if (after_null) (void)hipEventDestroy(after_null);
    if (st) (void)hipStreamDestroy(st);
  }
};

struct Program {
  int device = 0;
  uint32_t n_wires = 0, n_out = 0, n_pub = 0, n_prv = 0, n_levels = 0;
  DevBuf<Fr> consts, inv_small;
  DevBuf<DTerm> terms;
  DevBuf<Op> ops;
  DevBuf<Level> levels;
  // wire map of a remapped program (nzcb_wprog_remap): output wire t = program wire
  // wmap[t]; the program runs into a slot's scratch and a gather writes the target order
  uint32_t n_target = 0;
  DevBuf<uint32_t> wmap;
  std::mutex slot_mu;
  std::vector<std::unique_ptr<RunSlot>> slots;
  std::vector<RunSlot*> idle;
  uint32_t out_wires() const { return n_target ? n_target : n_wires; }
  RunSlot* acquire() {
    std::lock_guard<std::mutex> lk(slot_mu);
    if (idle.empty()) {
      slots.emplace_back(new RunSlot());
      NZ_HIP(hipStreamCreateWithFlags(&slots.back()->st, hipStreamNonBlocking));
      NZ_HIP(hipEventCreateWithFlags(&slots.back()->after_null, hipEventDisableTiming));
      return slots.back().get();
    }
    RunSlot* r = idle.back();
    idle.pop_back();
    return r;
  }
  void release(RunSlot* r) {
    std::lock_guard<std::mutex> lk(slot_mu);
    idle.push_back(r);
  }
};

// witness i, target wire t = scratch witness i, program wire map[t]
__global__ void __launch_bounds__(256)
wvm_gather_kernel(const Fr* __restrict__ src, size_t src_stride, const uint32_t* __restrict__ map, uint32_t T,
                  Fr* __restrict__ dst, size_t dst_stride) {
  const size_t i = blockIdx.y;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < T; t += (size_t)gridDim.x * blockDim.x)
    dst[i * dst_stride + t] = src[i * src_stride + map[t]];
}

// End offset of the input-names section (the program proper); throws on a malformed one
static size_t names_end(const uint8_t* data, size_t len, size_t need);

static uint32_t rd32(const uint8_t* p) {
  uint32_t x;
  std::memcpy(&x, p, 4);
  return x;
}

template <class T>
static void upload(DevBuf<T>& d, const void* src, size_t count) {
  d.alloc(count ? count : 1);
  if (count) NZ_HIP(hipMemcpy(d.p, src, count * sizeof(T), hipMemcpyHostToDevice));
}

Program* load(const uint8_t* data, size_t len, int device) {
  if (!data || len < 40 || std::memcmp(data, "nzwp", 4) != 0)
    throw Error(NZCB_ERR_FORMAT, "witness program: bad magic");
  if (rd32(data + 4) != 2) throw Error(NZCB_ERR_FORMAT, "witness program: unsupported version");
  auto P = new Program();
  try {
    P->device = device;
    P->n_wires = rd32(data + 8);
    P->n_out = rd32(data + 12);
    P->n_pub = rd32(data + 16);
    P->n_prv = rd32(data + 20);
    const uint32_t nc = rd32(data + 24), nt = rd32(data + 28), no = rd32(data + 32);
    P->n_levels = rd32(data + 36);
    const size_t need = 40 + (size_t)nc * 32 + (size_t)nt * 8 + (size_t)no * 32 + ((size_t)P->n_levels * 2 + 1) * 4;
    if (len < need + 4) throw Error(NZCB_ERR_FORMAT, "witness program: truncated");
    {  // input names (host-side mapping of input objects; checked here, not used on the GPU)
      size_t o = names_end(data, len, need);
      if (o != len) {  // optional wire map (nzcb_wprog_remap): "wmap" u32 T, T x u32
        if (o + 8 > len || std::memcmp(data + o, "wmap", 4) != 0)
          throw Error(NZCB_ERR_FORMAT, "witness program: oversized");
        const uint32_t T = rd32(data + o + 4);
        if (T == 0 || o + 8 + (size_t)T * 4 != len) throw Error(NZCB_ERR_FORMAT, "witness program: bad wire map");
        std::vector<uint32_t> m(T);
        std::memcpy(m.data(), data + o + 8, (size_t)T * 4);
        if (m[0] != 0) throw Error(NZCB_ERR_FORMAT, "witness program: wire map must keep wire 0");
        for (uint32_t t = 0; t < T; t++)
          if (m[t] >= P->n_wires) throw Error(NZCB_ERR_FORMAT, "witness program: wire map out of range");
        NZ_HIP(hipSetDevice(device));
        upload(P->wmap, m.data(), T);
        P->n_target = T;
      }
    }
    const uint8_t* p = data + 40;
    // coefficients c -> c R^2 (Montgomery of Montgomery), checked < r
    std::vector<Fr> cs(nc);
    std::vector<int32_t> sc(nc);
    for (uint32_t i = 0; i < nc; i++) {
      Fr c;
      std::memcpy(c.v, p + 32 * (size_t)i, 32);
      if (reduce_once(c) != c) throw Error(NZCB_ERR_FORMAT, "witness program: coefficient >= r");
      cs[i] = to_mont(to_mont(c));
      const Fr nc_ = neg(c);
      bool lo = true, nlo = true;
      for (int k = 1; k < 8; k++) {
        lo = lo && c.v[k] == 0;
        nlo = nlo && nc_.v[k] == 0;
      }
      if (lo && c.v[0] < 0x80000000u)
        sc[i] = (int32_t)c.v[0];
      else if (nlo && nc_.v[0] < 0x80000000u)
        sc[i] = -(int32_t)nc_.v[0];
      else
        sc[i] = kBigCoef;
    }
    p += (size_t)nc * 32;
    const Term* tm = (const Term*)p;
    for (uint32_t i = 0; i < nt; i++)
      if (tm[i].wire >= P->n_wires || tm[i].ci >= nc) throw Error(NZCB_ERR_FORMAT, "witness program: bad term");
    p += (size_t)nt * 8;
    const Op* op = (const Op*)p;
    for (uint32_t i = 0; i < no; i++) {
      const Op& o = op[i];
      const uint32_t typ = o.code & 0xFF, n = o.code >> 16;
      auto lc_ok = [&](uint32_t off, uint32_t cnt) { return (uint64_t)off + cnt <= nt; };
      bool ok = typ <= OP_SHA512;
      size_t width = 1;
      if (typ == OP_QUIN) {
        width = 2 * (size_t)n + o.b_n;
        ok = ok && lc_ok(o.a_off, o.a_n) && o.b_n <= n && (uint64_t)o.b_off + o.b_n <= P->n_wires;
      } else if (typ == OP_SHA256 || typ == OP_SHA512) {
        const size_t sz = typ == OP_SHA256 ? ShaLayout<32>::size : ShaLayout<64>::size;
        width = sz;
        ok = ok && (o.a_off == kNoWire || (uint64_t)o.a_off + sz <= P->n_wires) &&
             (uint64_t)o.b_off + 512 <= P->n_wires;
      } else {
        ok = ok && lc_ok(o.a_off, o.a_n) && lc_ok(o.b_off, o.b_n);
        if (typ != OP_BITS && typ != OP_CHECK) ok = ok && lc_ok(o.c_off, o.c_n);
        if (typ == OP_BITS) width = n;
        if (typ == OP_CHECK) width = 0;
        ok = ok && (typ != OP_BITS || (n >= 1 && n <= 254));
      }
      if (width) ok = ok && (uint64_t)o.dst + width <= P->n_wires;
      if (!ok) throw Error(NZCB_ERR_FORMAT, "witness program: bad op " + std::to_string(i));
    }
    p += (size_t)no * 32;
    const uint32_t* lv = (const uint32_t*)p;
    for (uint32_t i = 0; i < P->n_levels; i++) {
      const uint32_t s = lv[i], e = lv[i + 1], ms = lv[P->n_levels + 1 + i];
      if (!(s <= ms && ms <= e && e <= no)) throw Error(NZCB_ERR_FORMAT, "witness program: bad level table");
    }
    if (P->n_levels && lv[P->n_levels] != no) throw Error(NZCB_ERR_FORMAT, "witness program: bad level table");
    if (1 + P->n_out + P->n_pub + P->n_prv > P->n_wires) throw Error(NZCB_ERR_FORMAT, "witness program: bad counts");
    // 1/i for the small-integer fast path: one Fermat inverse and a prefix-product pass
    std::vector<Fr> pre(kInvTable), inv(kInvTable, Fr::zero());
    Fr acc = Fr::one();
    for (uint32_t i = 1; i < kInvTable; i++) {
      Fr fi = Fr::zero();
      fi.v[0] = i;
      pre[i] = acc;                 // prod_{k < i} k (Montgomery)
      acc = acc * to_mont(fi);
    }
    Fr ia = inverse(acc);           // 1 / prod_{k < T} k
    for (uint32_t i = kInvTable - 1; i >= 1; i--) {
      Fr fi = Fr::zero();
      fi.v[0] = i;
      inv[i] = from_mont(ia * pre[i]);
      ia = ia * to_mont(fi);
    }
    // each level's ops regrouped into its thread, wave and workgroup segments
    std::vector<Op> ro;
    ro.reserve(no);
    std::vector<Level> lt(P->n_levels);
    for (uint32_t i = 0; i < P->n_levels; i++) {
      const uint32_t s = lv[i], e = lv[i + 1];
      auto cls = [&](const Op& o) {  // 0 thread, 1 wave, 2 workgroup
        const uint32_t typ = o.code & 0xFF;
        if (typ == OP_SHA256 || typ == OP_SHA512) return 2;
        if (typ == OP_QUIN) return 1;
        uint32_t na, nb, nc;
        op_counts(o, na, nb, nc);
        return (uint64_t)na + nb + nc > kWaveTerms ? 1 : 0;
      };
      Level L;
      L.s = (uint32_t)ro.size();
      for (int c = 0; c < 3; c++) {
        if (c == 1) L.w = (uint32_t)ro.size();
        if (c == 2) L.m = (uint32_t)ro.size();
        for (uint32_t k = s; k < e; k++)
          if (cls(op[k]) == c) ro.push_back(op[k]);
      }
      L.e = (uint32_t)ro.size();
      lt[i] = L;
    }
    NZ_HIP(hipSetDevice(device));
    upload(P->consts, cs.data(), nc);
    std::vector<DTerm> dt(nt);
    for (uint32_t i = 0; i < nt; i++) dt[i] = DTerm{tm[i].wire, tm[i].ci, sc[tm[i].ci], 0};
    upload(P->terms, dt.data(), nt);
    upload(P->ops, ro.data(), no);
    upload(P->levels, lt.data(), P->n_levels);
    upload(P->inv_small, inv.data(), kInvTable);
  } catch (...) {
    delete P;
    throw;
  }
  return P;
}

static size_t names_end(const uint8_t* data, size_t len, size_t need) {
  size_t o = need;
  const uint32_t nn = rd32(data + o);
  o += 4;
  uint64_t total = 0;
  for (uint32_t i = 0; i < nn; i++) {
    if (o + 4 > len) throw Error(NZCB_ERR_FORMAT, "witness program: truncated input names");
    const uint32_t ln = rd32(data + o);
    o += 4 + (size_t)ln;
    if (o + 4 > len) throw Error(NZCB_ERR_FORMAT, "witness program: truncated input names");
    total += rd32(data + o);
    o += 4;
  }
  if (o > len) throw Error(NZCB_ERR_FORMAT, "witness program: truncated input names");
  if (nn && total != (uint64_t)rd32(data + 16) + rd32(data + 20))
    throw Error(NZCB_ERR_FORMAT, "witness program: input names do not cover the inputs");
  return o;
}

void run(Program* P, const void* dev_inputs, int count, void* dev_witness, size_t stride_bytes, int32_t* status_out,
         hipStream_t s) {
  if (count <= 0) return;
  if (!dev_inputs || !dev_witness || !status_out) throw Error(NZCB_ERR_ARG, "witness program: null buffer");
  if (stride_bytes % 32 || stride_bytes < (size_t)P->out_wires() * 32)
    throw Error(NZCB_ERR_ARG, "witness program: witness stride below n_wires x 32 B");
  NZ_HIP(hipSetDevice(P->device));
  RunSlot* R = P->acquire();
  struct Release {
    Program* P;
    RunSlot* R;
    ~Release() { P->release(R); }
  } release{P, R};
  if (!s) {  // no stream given: the slot's, after whatever the caller queued on the null stream
    NZ_HIP(hipEventRecord(R->after_null, nullptr));
    NZ_HIP(hipStreamWaitEvent(R->st, R->after_null, 0));
    s = R->st;
  }
  Fr* run_dst = (Fr*)dev_witness;
  size_t run_stride = stride_bytes / 32;
  if (P->n_target) {  // remapped: the program's own wire order into scratch, then the gather
    if ((size_t)count > R->scratch_cap) {
      R->scratch.alloc((size_t)count * P->n_wires);
      R->scratch_cap = (size_t)count;
    }
    run_dst = R->scratch.p;
    run_stride = P->n_wires;
  }
  if ((size_t)count > R->status_cap) {
    R->status.alloc((size_t)count);
    R->status_cap = (size_t)count;
  }
  Prog g;
  g.consts = P->consts.p;
  g.terms = P->terms.p;
  g.ops = P->ops.p;
  g.levels = P->levels.p;
  g.inv_small = P->inv_small.p;
  g.n_levels = P->n_levels;
  g.n_wires = P->n_wires;
  g.n_inputs = P->n_pub + P->n_prv;
  g.in_base = 1 + P->n_out;
  // NZCB_WVM_LEVEL_CLOCK=<file>: pass 0's wall clocks per level (kClockSlots u64 ticks
  // each, level 0 = kernel start), appended to <file> (tools/wvm_bench.py; off by default)
  const char* clock_path = std::getenv("NZCB_WVM_LEVEL_CLOCK");
  DevBuf<uint64_t> lclk;
  if (clock_path && *clock_path) {
    lclk.alloc(((size_t)P->n_levels + 1) * kClockSlots);
    NZ_HIP(hipMemsetAsync(lclk.p, 0, ((size_t)P->n_levels + 1) * kClockSlots * 8, s));
  }
  hipLaunchKernelGGL(wvm_kernel<kWvmThreads>, dim3((unsigned)count), dim3(kWvmThreads), 0, s, g,
                     (const Fr*)dev_inputs, run_dst, run_stride, R->status.p, lclk.p);
  NZ_HIP(hipGetLastError());
  if (P->n_target) {
    const unsigned gx = (unsigned)std::min<size_t>(((size_t)P->n_target + 255) / 256, 1024);
    hipLaunchKernelGGL(wvm_gather_kernel, dim3(gx, (unsigned)count), dim3(256), 0, s, (const Fr*)run_dst,
                       run_stride, P->wmap.p, P->n_target, (Fr*)dev_witness, stride_bytes / 32);
    NZ_HIP(hipGetLastError());
  }
  std::vector<uint32_t> st((size_t)count);
  NZ_HIP(hipMemcpyAsync(st.data(), R->status.p, (size_t)count * 4, hipMemcpyDeviceToHost, s));
  NZ_HIP(hipStreamSynchronize(s));
  if (lclk.p) {
    std::vector<uint64_t> h(((size_t)P->n_levels + 1) * kClockSlots, 0);
    NZ_HIP(hipMemcpy(h.data(), lclk.p, h.size() * 8, hipMemcpyDeviceToHost));
    if (FILE* f = std::fopen(clock_path, "ab")) {
      std::fwrite(h.data(), 8, h.size(), f);
      std::fclose(f);
    }
  }
  for (int i = 0; i < count; i++) status_out[i] = st[i] == 0xFFFFFFFFu ? 0 : (int32_t)(st[i] & 0xFF);
}

}  // namespace wvm
}  // namespace nzcb

using namespace nzcb;

struct nzcb_wprog {
  wvm::Program* p;  // concurrent runs take a RunSlot each (no lock around a run)
};

extern "C" {

nzcb_wprog* nzcb_wprog_create(const uint8_t* prog, size_t len, int device, nzcb_err* err) {
  try {
    auto h = new nzcb_wprog();
    try {
      h->p = wvm::load(prog, len, device);
    } catch (...) {
      delete h;
      throw;
    }
    return h;
  } catch (const Error& e) {
    set_err(err, e.code, e.what());
  } catch (const std::exception& e) {
    set_err(err, NZCB_ERR_INTERNAL, e.what());
  }
  return nullptr;
}

void nzcb_wprog_destroy(nzcb_wprog* h) {
  if (!h) return;
  if (h->p) {
    (void)hipSetDevice(h->p->device);
    delete h->p;
  }
  delete h;
}

int nzcb_wprog_info(const nzcb_wprog* h, uint32_t info[5]) {
  if (!h || !info) return NZCB_ERR_ARG;
  info[0] = h->p->out_wires();
  info[1] = h->p->n_out;
  info[2] = h->p->n_pub;
  info[3] = h->p->n_prv;
  info[4] = h->p->n_levels;
  return NZCB_OK;
}

int nzcb_wprog_run_dev(nzcb_wprog* h, const void* dev_inputs, int count, void* dev_witness, size_t witness_stride,
                       int32_t* status_out, void* stream, nzcb_err* err) {
  try {
    if (!h) throw Error(NZCB_ERR_ARG, "witness program: null handle");
    wvm::run(h->p, dev_inputs, count, dev_witness, witness_stride, status_out, (hipStream_t)stream);
    return NZCB_OK;
  } catch (const Error& e) {
    set_err(err, e.code, e.what());
    return e.code;
  } catch (const std::exception& e) {
    set_err(err, NZCB_ERR_INTERNAL, e.what());
    return NZCB_ERR_INTERNAL;
  }
}

int nzcb_wprog_run(nzcb_wprog* h, const uint8_t* inputs, int count, uint8_t* witness_out, int32_t* status_out,
                   nzcb_err* err) {
  try {
    if (!h) throw Error(NZCB_ERR_ARG, "witness program: null handle");
    if (count <= 0) return NZCB_OK;
    if (!inputs || !witness_out || !status_out) throw Error(NZCB_ERR_ARG, "witness program: null buffer");
    NZ_HIP(hipSetDevice(h->p->device));
    const size_t nin = (size_t)(h->p->n_pub + h->p->n_prv) * 32 * count;
    const size_t nw = (size_t)h->p->out_wires() * 32;
    DevBuf<uint8_t> din(nin ? nin : 1), dw(nw * count);
    if (nin) NZ_HIP(hipMemcpy(din.p, inputs, nin, hipMemcpyHostToDevice));
    wvm::run(h->p, din.p, count, dw.p, nw, status_out, nullptr);
    NZ_HIP(hipMemcpy(witness_out, dw.p, nw * count, hipMemcpyDeviceToHost));
    return NZCB_OK;
  } catch (const Error& e) {
    set_err(err, e.code, e.what());
    return e.code;
  } catch (const std::exception& e) {
    set_err(err, NZCB_ERR_INTERNAL, e.what());
    return NZCB_ERR_INTERNAL;
  }
}

// circom .sym text: "label,wire,component,name" per line; wire < 0 = optimized out
static void parse_sym(const char* text, size_t len,
                      const std::function<void(int64_t wire, const std::string& name)>& f) {
  size_t o = 0;
  while (o < len) {
    size_t e = o;
    while (e < len && text[e] != '\n') e++;
    std::string line(text + o, e - o);
    o = e + 1;
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (line.empty()) continue;
    const size_t c1 = line.find(','), c2 = c1 == std::string::npos ? c1 : line.find(',', c1 + 1),
                 c3 = c2 == std::string::npos ? c2 : line.find(',', c2 + 1);
    if (c3 == std::string::npos) throw Error(NZCB_ERR_FORMAT, "sym: malformed line: " + line.substr(0, 80));
    char* end = nullptr;
    const std::string ws = line.substr(c1 + 1, c2 - c1 - 1);
    const long long wire = std::strtoll(ws.c_str(), &end, 10);
    if (!end || *end) throw Error(NZCB_ERR_FORMAT, "sym: bad wire index: " + line.substr(0, 80));
    f(wire, line.substr(c3 + 1));
  }
}

int nzcb_wprog_remap(const uint8_t* prog, size_t len, const char* own_sym, size_t own_len, const char* target_sym,
                     size_t target_len, uint8_t** out, size_t* out_len, uint32_t* unmatched, nzcb_err* err) {
  try {
    if (!prog || !own_sym || !target_sym || !out || !out_len) throw Error(NZCB_ERR_ARG, "null argument");
    if (unmatched) *unmatched = 0;
    if (len < 40 || std::memcmp(prog, "nzwp", 4) != 0) throw Error(NZCB_ERR_FORMAT, "witness program: bad magic");
    const uint32_t n_wires = wvm::rd32(prog + 8), nc = wvm::rd32(prog + 24), nt = wvm::rd32(prog + 28),
                   no = wvm::rd32(prog + 32), nl = wvm::rd32(prog + 36);
    const size_t need = 40 + (size_t)nc * 32 + (size_t)nt * 8 + (size_t)no * 32 + ((size_t)nl * 2 + 1) * 4;
    if (len < need + 4) throw Error(NZCB_ERR_FORMAT, "witness program: truncated");
    if (wvm::names_end(prog, len, need) != len)
      throw Error(NZCB_ERR_FORMAT, "witness program: already remapped (or oversized)");
    std::unordered_map<std::string, uint32_t> own;
    own.reserve(n_wires);
    parse_sym(own_sym, own_len, [&](int64_t wire, const std::string& name) {
      if (wire >= 0) {
        if (wire >= n_wires) throw Error(NZCB_ERR_FORMAT, "sym: wire beyond the program's: " + name);
        own.emplace(name, (uint32_t)wire);
      }
    });
    std::vector<std::vector<std::string>> names;  // target wire -> its names
    parse_sym(target_sym, target_len, [&](int64_t wire, const std::string& name) {
      if (wire < 0) return;
      if (wire >= (1ll << 31)) throw Error(NZCB_ERR_FORMAT, "sym: wire index too large");
      if ((size_t)wire >= names.size()) names.resize((size_t)wire + 1);
      names[(size_t)wire].push_back(name);
    });
    const uint32_t T = names.size() ? (uint32_t)names.size() : 1;
    std::vector<uint32_t> map(T, 0);
    uint32_t miss = 0;
    std::string first;
    for (uint32_t t = 1; t < T; t++) {
      bool ok = false;
      for (const auto& nm : names[t]) {
        auto it = own.find(nm);
        if (it != own.end()) {
          map[t] = it->second;
          ok = true;
          break;
        }
      }
      if (!ok) {
        if (!miss) first = names[t].empty() ? "(wire " + std::to_string(t) + " has no name)" : names[t][0];
        miss++;
      }
    }
    if (unmatched) *unmatched = miss;
    if (miss)
      throw Error(NZCB_ERR_FORMAT, std::to_string(miss) + " of " + std::to_string(T - 1) +
                                       " target signals have no counterpart in the program, e.g. " + first);
    const size_t total = len + 8 + (size_t)T * 4;
    uint8_t* buf = (uint8_t*)std::malloc(total);
    if (!buf) throw Error(NZCB_ERR_INTERNAL, "out of host memory");
    std::memcpy(buf, prog, len);
    std::memcpy(buf + len, "wmap", 4);
    std::memcpy(buf + len + 4, &T, 4);
    std::memcpy(buf + len + 8, map.data(), (size_t)T * 4);
    *out = buf;
    *out_len = total;
    return NZCB_OK;
  } catch (const Error& e) {
    set_err(err, e.code, e.what());
    return e.code;
  } catch (const std::exception& e) {
    set_err(err, NZCB_ERR_INTERNAL, e.what());
    return NZCB_ERR_INTERNAL;
  }
}

}  // extern "C"
