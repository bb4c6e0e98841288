// nzcp witness kernel: the semantic signals and public outputs of the nzcp circuit
// NZCPPubIdentity (/root/reference/circuits/nzcptpl.circom:444-655) for a batch of
// passes, one workgroup per pass. It replaces the part of
// circom_runtime's WitnessCalculator.calculateWitness(input, sanityCheck) [EXT] that
// the prover's public inputs depend on: the input bit checks, Sha256Var over the
// ToBeSigned, the CBOR/CWT scan (cbortpl.circom), the nullifier concat, Sha512 and
// the 3 x 248-bit output packing. The CPU restatement it is checked against is
// oracle/nzcp_circuit.py; gadget order, range checks and error codes follow it
// line for line (the first failing check in template order is reported).
//
// Work split per pass (256 threads):
//   phase A  all waves: coalesced read of the (MaxToBeSignedBytes*8 + 161) input
//            signals (32-byte LE field elements), bit checks, bits -> bytes with one
//            wave ballot per 64 signals, the data term sum_j data_j * 2^(40+j) mod r
//   phase B  wave 0 lane 0: SHA-256 of ToBeSigned[0, len)
//            wave 1 lane 0: CBOR scan -> credential subject -> nullifier -> SHA-512
//            (two waves, so both serial chains issue concurrently)
//   phase C  thread 0: output packing, record, optional public-signal write into a
//            device witness (witness[1..3]) for the prover.
// Input traffic dominates HBM: (8*MaxBytes + 161) * 32 B per pass (95 KB live).
#include <climits>
#include <cstring>
#include <vector>

#include "../../include/nzcb.h"
#include "common.h"
#include "engine.h"

namespace nzcb {
namespace nzcp {

constexpr int kThreads = 256;
constexpr int kMaxBytes = 512;     // ToBeSignedBlockSpace = 3: 8 blocks of 512 bits
constexpr int kMaxArray = 8;       // MaxCborArrayLen supported by SkipValue here
constexpr int kMaxMap = 32;        // MaxCborMapLen supported by FindCWTClaims here
constexpr int kNullifier = 64;     // NULLIFIFER_BYTES
constexpr int kMaxStr = kNullifier / 3;  // ReadCredSubj MaxStringLen = 21
constexpr int kData = 160;

enum { kMajorInt = 0, kMajorString = 3, kMajorArray = 4, kMajorMap = 5 };

__device__ __forceinline__ int32_t clamp32(int64_t x) {
  return x < INT_MIN ? INT_MIN : (x > INT_MAX ? INT_MAX : (int32_t)x);
}

__device__ __forceinline__ int ilog2f(int64_t x) {  // log2.circom:5-12 (floor, log2(0) = -1)
  int z = -1;
  while (x) { z++; x /= 2; }
  return z;
}

// One lane's evaluation of the CBOR part. Errors never stop the evaluation (every
// read is bounds-guarded); the first one is kept, which is the circuit's first
// failing check because the evaluation order is the template order.
struct Scan {
  const uint8_t* bs;  // LDS, masked ToBeSigned bytes
  int n;              // MaxToBeSignedBytes
  int code = NZCB_NZCP_OK;
  int32_t detail = 0;

  __device__ void fail(int c, int64_t d) {
    if (code == NZCB_NZCP_OK) { code = c; detail = clamp32(d); }
  }
  // circomlib LessThan(nb): Num2Bits(nb+1) of a + 2^nb - b
  __device__ int64_t lt(int nb, int64_t a, int64_t b) {
    int64_t t = a + ((int64_t)1 << nb) - b;
    if (t < 0 || t >= ((int64_t)1 << (nb + 1))) { fail(NZCB_NZCP_ERR_RANGE, a); return 0; }
    return t < ((int64_t)1 << nb) ? 1 : 0;
  }
  // QuinSelector(choices) range rule: index in [choices - 2^bits, choices)
  __device__ bool sel_ok(int choices, int64_t index) {
    int bits = ilog2f(choices) + 1;
    int64_t t = index + ((int64_t)1 << bits) - choices;
    if (t < 0 || t >= ((int64_t)1 << bits)) { fail(NZCB_NZCP_ERR_SELECT, index); return false; }
    return index >= 0 && index < choices;
  }
  __device__ int64_t get_v(int64_t pos) { return sel_ok(n, pos) ? (int64_t)bs[pos] : 0; }
  __device__ int64_t byte_check(int64_t v) {
    if (v < 0 || v > 255) fail(NZCB_NZCP_ERR_RANGE, v);
    return v;
  }
  __device__ int64_t get_x(int64_t v) { return byte_check(v) & 31; }
  __device__ int64_t get_type(int64_t v) { return byte_check(v) >> 5; }

  __device__ int64_t decode_uint23(int64_t v) {  // cbortpl.circom:93-114
    int64_t x = get_x(v);
    if (lt(8, x, 24) != 1) fail(NZCB_NZCP_ERR_UINT23, x);
    return x;
  }
  // DecodeUint (cbortpl.circom:116-237): value, nextPos; every GetV is evaluated
  __device__ void decode_uint(int64_t pos, int64_t v, int64_t& value, int64_t& next) {
    int64_t x = get_x(v);
    int64_t c23 = lt(8, x, 24);
    int64_t c24 = x == 24, c25 = x == 25, c26 = x == 26;
    int64_t v24 = get_v(c24 * pos);
    int64_t v1_25 = get_v(c25 * pos);
    int64_t v2_25 = get_v(c25 * (pos + 1));
    int64_t v1_26 = get_v(c26 * pos);
    int64_t v2_26 = get_v(c26 * (pos + 1));
    int64_t v3_26 = get_v(c26 * (pos + 2));
    int64_t v4_26 = get_v(c26 * (pos + 3));
    value = c23 * x + c24 * v24 + c25 * (v1_25 * 256 + v2_25) +
            c26 * (v1_26 * 16777216 + v2_26 * 65536 + v3_26 * 256 + v4_26);
    next = c23 * pos + c24 * (pos + 1) + c25 * (pos + 2) + c26 * (pos + 4);
  }
  __device__ void read_type(int64_t pos, int64_t& next, int64_t& type, int64_t& v) {
    v = get_v(pos);
    type = get_type(v);
    next = pos + 1;
  }
  __device__ int64_t skip_value_scalar(int64_t pos) {  // cbortpl.circom:264-297
    int64_t nt, t, v, value, np;
    read_type(pos, nt, t, v);
    decode_uint(nt, v, value, np);
    return (t == kMajorInt) * np + (t == kMajorString) * (np + value);
  }
  __device__ int64_t skip_value(int64_t pos, int max_arr) {  // cbortpl.circom:300-360
    int64_t nt, t, v, value, np;
    read_type(pos, nt, t, v);
    decode_uint(nt, v, value, np);
    int64_t is_int = t == kMajorInt, is_str = t == kMajorString, is_arr = t == kMajorArray;
    int64_t nexts[kMaxArray];
    int bits = ilog2f(max_arr) + 1;
    for (int i = 0; i < max_arr; i++) {
      int64_t consider = is_arr * lt(bits, i, is_arr * value);
      int64_t p = (i == 0 ? np : nexts[i - 1]) * consider;
      nexts[i] = skip_value_scalar(p);
    }
    int64_t qs = 0;
    if (max_arr > 0) {
      int64_t idx = is_arr * (value - 1);
      if (sel_ok(max_arr, idx)) {
        for (int i = 0; i < max_arr; i++)
          if (i == idx) qs = nexts[i];
      }
    }
    return is_int * np + is_str * (np + value) + is_arr * qs;
  }
  template <int L>
  __device__ int64_t string_equals(int64_t pos, int64_t len, const char (&c)[L]) {  // :362-400
    constexpr int n_c = L - 1;
    int64_t s = len == n_c;
    for (int i = 0; i < n_c; i++) s += ((int64_t)(uint8_t)c[i] == get_v(pos + i));
    return (n_c + 1 - s) == 0;
  }
  __device__ void read_string_length(int64_t pos, int64_t& len, int64_t& next) {  // :402-425
    int64_t nt, t, v, np;
    read_type(pos, nt, t, v);
    if (t != kMajorString) fail(NZCB_NZCP_ERR_NOT_STRING, pos);
    decode_uint(nt, v, len, np);
    next = nt;
  }
  __device__ void read_map_length(int64_t pos, int64_t& len, int64_t& next) {  // :427-451
    int64_t nt, t, v;
    read_type(pos, nt, t, v);
    if (t != kMajorMap) fail(NZCB_NZCP_ERR_NOT_MAP, pos);
    len = decode_uint23(v);
    next = nt;
  }
  // CopyString(n, kMaxStr) (cbortpl.circom:453-503) into out[0..kMaxStr)
  __device__ void copy_string(int64_t pos, int32_t* out, int64_t& next, int64_t& len) {
    int64_t np;
    read_string_length(pos, len, np);
    constexpr int bits = 5;  // log2(21) + 1
    for (int i = 0; i < kMaxStr; i++) {
      int64_t b = get_v(np + i);
      out[i] = (int32_t)(b * lt(bits, i, len));
    }
    next = np + len;
  }
};

struct Shared {
  uint8_t raw[kMaxBytes];         // ToBeSigned bytes, masked past len after phase A
  Fr data_terms[kData];
  int32_t copies[3][kMaxStr];
  int32_t names[3][kNullifier];   // given, family, dob (ReadCredSubj outputs)
  int32_t result[kNullifier];     // ConstructNullifier.result before its Num2Bits(8)
  uint8_t nullifier[kNullifier];
  uint8_t sha256[32];
  uint8_t sha512[64];
  int bad_bit;
  int code;
  int32_t detail;
  uint32_t exp;
  int32_t vc_pos, lens[3], null_len;
};

// ---- SHA-256 / SHA-512 (FIPS 180-4) -------------------------------------------
__constant__ uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__constant__ uint64_t K512[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

__device__ __forceinline__ uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
__device__ __forceinline__ uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

// SHA-256 of msg[0, len) (len < 2^29), digest big-endian into out[32]
__device__ void sha256(const uint8_t* msg, int len, uint8_t* out) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  int nblocks = (len + 9 + 63) / 64;
  uint64_t bitlen = (uint64_t)len * 8;
  for (int blk = 0; blk < nblocks; blk++) {
    uint32_t w[16];
#pragma unroll
    for (int t = 0; t < 16; t++) {
      uint32_t word = 0;
#pragma unroll
      for (int b = 0; b < 4; b++) {
        int idx = blk * 64 + 4 * t + b;
        uint32_t byte = idx < len ? msg[idx] : (idx == len ? 0x80u : 0u);
        if (blk == nblocks - 1 && t >= 14) byte = (uint32_t)(bitlen >> (8 * (7 - (4 * (t - 14) + b)))) & 0xffu;
        word = (word << 8) | byte;
      }
      w[t] = word;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
    for (int i = 0; i < 64; i++) {
      uint32_t wi;
      if (i < 16) {
        wi = w[i];
      } else {
        uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
        uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
        uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
        wi = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
        w[i & 15] = wi;
      }
      uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
      uint32_t ch = (e & f) ^ (~e & g);
      uint32_t t1 = hh + S1 + ch + K256[i] + wi;
      uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
      uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
      uint32_t t2 = S0 + mj;
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
#pragma unroll
  for (int i = 0; i < 8; i++)
#pragma unroll
    for (int b = 0; b < 4; b++) out[4 * i + b] = (uint8_t)(h[i] >> (24 - 8 * b));
}

// SHA-512 of a 64-byte message (Sha512(512)): one padded block
__device__ void sha512_64(const uint8_t* msg, uint8_t* out) {
  uint64_t h[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                   0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  uint64_t w[16];
#pragma unroll
  for (int t = 0; t < 8; t++) {
    uint64_t x = 0;
#pragma unroll
    for (int b = 0; b < 8; b++) x = (x << 8) | msg[8 * t + b];
    w[t] = x;
  }
  w[8] = 0x8000000000000000ULL;
#pragma unroll
  for (int t = 9; t < 15; t++) w[t] = 0;
  w[15] = 512;
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int i = 0; i < 80; i++) {
    uint64_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint64_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      uint64_t s0 = rotr64(w15, 1) ^ rotr64(w15, 8) ^ (w15 >> 7);
      uint64_t s1 = rotr64(w2, 19) ^ rotr64(w2, 61) ^ (w2 >> 6);
      wi = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
      w[i & 15] = wi;
    }
    uint64_t S1 = rotr64(e, 14) ^ rotr64(e, 18) ^ rotr64(e, 41);
    uint64_t ch = (e & f) ^ (~e & g);
    uint64_t t1 = hh + S1 + ch + K512[i] + wi;
    uint64_t S0 = rotr64(a, 28) ^ rotr64(a, 34) ^ rotr64(a, 39);
    uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint64_t t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
#pragma unroll
  for (int i = 0; i < 8; i++)
#pragma unroll
    for (int b = 0; b < 8; b++) out[8 * i + b] = (uint8_t)(h[i] >> (56 - 8 * b));
}

// ---- field input helpers ----------------------------------------------------------
__device__ __forceinline__ Fr load_reduced(const uint8_t* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 lo = q[0], hi = q[1];
  Fr x;
  x.v[0] = lo.x; x.v[1] = lo.y; x.v[2] = lo.z; x.v[3] = lo.w;
  x.v[4] = hi.x; x.v[5] = hi.y; x.v[6] = hi.z; x.v[7] = hi.w;
  for (int k = 0; k < 6; k++) x = reduce_once(x);  // any 256-bit value < 6r
  return x;
}

// field element -> signed int64, saturated to +-2^62 (enough for every range check)
__device__ int64_t field_signed(const Fr& x) {
  const int64_t sat = (int64_t)1 << 62;
  bool small = x.v[7] == 0 && x.v[6] == 0 && x.v[5] == 0 && x.v[4] == 0 && x.v[3] == 0 && x.v[2] == 0 &&
               x.v[1] < (1u << 30);
  if (small) return (int64_t)(((uint64_t)x.v[1] << 32) | x.v[0]);
  Fr y = neg(x);  // r - x
  bool small_neg = y.v[7] == 0 && y.v[6] == 0 && y.v[5] == 0 && y.v[4] == 0 && y.v[3] == 0 && y.v[2] == 0 &&
                   y.v[1] < (1u << 30);
  if (small_neg) return -(int64_t)(((uint64_t)y.v[1] << 32) | y.v[0]);
  // |x| >= 2^62 either way: x > r/2 reads as negative (oracle _field_signed)
  const uint32_t HALF[8] = {0xf8000000u, 0xa1f0fac9u, 0x3cdcb848u, 0x9419f424u,
                            0x40c0ac2eu, 0xdc2822dbu, 0x7098d014u, 0x18322739u};
  for (int i = 7; i >= 0; i--) {
    if (x.v[i] != HALF[i]) return x.v[i] > HALF[i] ? -sat : sat;
  }
  return sat;
}

__device__ void store_fr_le(uint8_t* dst, const Fr& x) {
  for (int i = 0; i < 8; i++)
    for (int b = 0; b < 4; b++) dst[4 * i + b] = (uint8_t)(x.v[i] >> (8 * b));
}

// big-endian bytes -> Fr (value < 2^248)
__device__ Fr fr_from_be31(const uint8_t* be) {
  Fr x = Fr::zero();
  for (int k = 0; k < 31; k++) {
    int bit = 8 * (30 - k);
    x.v[bit / 32] |= (uint32_t)be[k] << (bit % 32);
  }
  return x;
}

__global__ __launch_bounds__(kThreads) void nzcp_witness_kernel(const uint8_t* __restrict__ inputs, int count,
                                                                 nzcb_nzcp_params prm,
                                                                 nzcb_nzcp_record* __restrict__ records,
                                                                 uint8_t* __restrict__ witness, size_t wit_stride) {
  __shared__ Shared sh;
  const int pass = blockIdx.x;
  if (pass >= count) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n_bytes = prm.max_tbs_bytes;
  const int n_bits = n_bytes * 8;
  const size_t n_in = (size_t)n_bits + 1 + kData;
  const uint8_t* in = inputs + (size_t)pass * n_in * 32;

  if (tid == 0) sh.bad_bit = INT_MAX;
  for (int k = tid; k < kMaxBytes; k += kThreads) sh.raw[k] = 0;
  __syncthreads();

  // phase A: bits (nzcptpl.circom:493-496, 521-533) ...
  for (int base = wave * 64; base < n_bits; base += kThreads) {
    int i = base + lane;
    int bit = 0;
    if (i < n_bits) {
      Fr x = load_reduced(in + (size_t)i * 32);
      bool hi0 = (x.v[1] | x.v[2] | x.v[3] | x.v[4] | x.v[5] | x.v[6] | x.v[7]) == 0;
      if (!hi0 || x.v[0] > 1) atomicMin(&sh.bad_bit, i);
      bit = (hi0 && x.v[0] == 1) ? 1 : 0;
    }
    uint64_t mask = __ballot(bit);
    if (lane < 8) {
      int byte = base / 8 + lane;
      if (byte < n_bytes) sh.raw[byte] = __builtin_bitreverse8((uint8_t)(mask >> (8 * lane)));
    }
  }
  // ... the data term (Bits2Num into out[2] at bit 40 + j, :626-650), any field values
  if (tid < kData) {
    Fr x = load_reduced(in + ((size_t)n_bits + 1 + tid) * 32);
    Fr pw = Fr::zero();
    pw.v[(40 + tid) / 32] = 1u << ((40 + tid) % 32);
    sh.data_terms[tid] = x * (pw * Fr::r2());  // x * 2^(40+j) in normal form
  }
  // ... and toBeSignedLen (:500-505); every thread evaluates it (broadcast read)
  const int64_t len = field_signed(load_reduced(in + (size_t)n_bits * 32));
  __syncthreads();

  int code = NZCB_NZCP_OK;
  int32_t detail = 0;
  if (sh.bad_bit != INT_MAX) {
    code = NZCB_NZCP_ERR_BIT;
    detail = sh.bad_bit;
  } else {
    Scan s;
    s.bs = sh.raw;
    s.n = n_bytes;
    int bits = ilog2f(n_bytes + 1) + 1;
    if (s.lt(bits, len, n_bytes + 1) != 1) s.fail(NZCB_NZCP_ERR_LEN, len);
    if (s.code == NZCB_NZCP_OK && len < 0) s.fail(NZCB_NZCP_ERR_UNPINNED, len);
    code = s.code;
    detail = s.detail;
  }
  if (code == NZCB_NZCP_OK) {  // ToBeSigned[k] = byte * (k < len)  (lt never fails for 0 <= len <= n)
    for (int k = tid; k < n_bytes; k += kThreads)
      if (k >= len) sh.raw[k] = 0;
  }
  __syncthreads();

  // phase B
  if (code == NZCB_NZCP_OK) {
    if (tid == 0) {
      sha256(sh.raw, (int)len, sh.sha256);  // Sha256Var(3), :509-517
    } else if (tid == 64) {
      Scan s;
      s.bs = sh.raw;
      s.n = n_bytes;
      // ReadMapLength at ClaimsSkip, :535-538
      int64_t map_len, pos;
      s.read_map_length(prm.is_live ? 30 : 27, map_len, pos);
      // FindCWTClaims, :28-145 / :540-546
      int64_t vc_pos = 0, exp_pos = 0, p = pos;
      for (int k = 0; k < prm.max_map_len_vc; k++) {
        int64_t nt, t, v, value, np;
        s.read_type(p, nt, t, v);
        s.decode_uint(nt, v, value, np);
        int64_t is_str = t == kMajorString, is_int = t == kMajorInt;
        int64_t p_next = s.skip_value(np + value * is_str, prm.max_array_len_vc);
        int64_t needle = s.string_equals(np, value, "vc");
        int64_t is4 = value == 4;
        int64_t within = s.lt(8, k, map_len);
        vc_pos += is_str * needle * within * (np + value);
        exp_pos += is_int * is4 * within * np;
        p = p_next;
      }
      int64_t exp, nt, t, v, np;
      s.read_type(exp_pos, nt, t, v);
      s.decode_uint(nt, v, exp, np);
      // ReadCredSubj(n, 64) at 171 + vcPos, :232-380 / :548-552
      int64_t flags[3][3];
      int64_t clen[3];
      p = 171 + vc_pos;
      for (int k = 0; k < 3; k++) {
        int64_t slen, np2;
        s.read_string_length(p, slen, np2);
        flags[k][0] = s.string_equals(np2, slen, "givenName");
        flags[k][1] = s.string_equals(np2, slen, "familyName");
        flags[k][2] = s.string_equals(np2, slen, "dob");
        s.copy_string(np2 + slen, sh.copies[k], p, clen[k]);
      }
      int64_t lens[3];
      for (int which = 0; which < 3; which++) {
        for (int h = 0; h < kNullifier; h++) {
          int64_t c = 0;
          if (h < kMaxStr)
            for (int k = 0; k < 3; k++) c += flags[k][which] * sh.copies[k][h];
          sh.names[which][h] = (int32_t)c;
        }
        lens[which] = flags[0][which] * clen[0] + flags[1][which] * clen[1] + flags[2][which] * clen[2];
      }
      // ConstructNullifier(64), :382-433 / :554-563
      const int64_t gl = lens[0], fl = lens[1], dl = lens[2];
      constexpr int nb = 7;  // log2(64) + 1
      for (int k = 0; k < kNullifier; k++) {
        int64_t is_g = s.lt(nb, k, gl);
        int64_t u_sep1 = s.lt(nb, k, gl + 1);
        int64_t u_fam = s.lt(nb, k, gl + 1 + fl);
        int64_t u_sep2 = s.lt(nb, k, gl + 1 + fl + 1);
        int64_t gs = s.sel_ok(kNullifier, k) ? sh.names[0][k] : 0;
        int64_t fi = k - gl - 1, di = k - gl - 1 - fl - 1;
        int64_t fs = s.sel_ok(kNullifier, fi) ? sh.names[1][fi] : 0;
        int64_t ds = s.sel_ok(kNullifier, di) ? sh.names[2][di] : 0;
        int64_t sep1 = u_sep1 * (1 - is_g), fam = u_fam * (1 - u_sep1), sep2 = u_sep2 * (1 - u_fam);
        int64_t is_d = 1 - u_sep2;
        sh.result[k] = clamp32(is_g * gs + sep1 * 44 + fam * fs + sep2 * 44 + is_d * ds);
      }
      for (int k = 0; k < kNullifier; k++) sh.nullifier[k] = (uint8_t)s.byte_check(sh.result[k]);  // Num2Bits(8), :566-573
      if (exp < 0 || exp >= ((int64_t)1 << 32)) s.fail(NZCB_NZCP_ERR_RANGE, exp);  // Num2Bits(32), :583-584
      sha512_64(sh.nullifier, sh.sha512);  // Sha512(512), :577-580
      sh.code = s.code;
      sh.detail = s.detail;
      sh.exp = (uint32_t)exp;
      sh.vc_pos = clamp32(vc_pos);
      sh.lens[0] = clamp32(gl);
      sh.lens[1] = clamp32(fl);
      sh.lens[2] = clamp32(dl);
      sh.null_len = clamp32(gl + 1 + fl + 1 + dl);
    }
  }
  __syncthreads();

  // phase C: packing (:586-654) and the record
  if (tid != 0) return;
  if (code == NZCB_NZCP_OK) {
    code = sh.code;
    detail = sh.detail;
  }
  nzcb_nzcp_record rec;
  memset(&rec, 0, sizeof(rec));
  rec.status = code;
  rec.detail = detail;
  if (code == NZCB_NZCP_OK) {
    uint8_t w[31];
    Fr out[3];
    for (int k = 0; k < 31; k++) w[k] = sh.sha512[k];
    out[0] = fr_from_be31(w);
    w[0] = sh.sha512[31];
    for (int k = 1; k < 31; k++) w[k] = sh.sha256[k - 1];
    out[1] = fr_from_be31(w);
    for (int k = 0; k < 31; k++) w[k] = 0;
    w[0] = sh.sha256[30];
    w[1] = sh.sha256[31];
    for (int k = 0; k < 4; k++) w[2 + k] = (uint8_t)(sh.exp >> (24 - 8 * k));
    Fr o2 = fr_from_be31(w);
    for (int j = 0; j < kData; j++) o2 = o2 + sh.data_terms[j];
    out[2] = o2;
    rec.exp = sh.exp;
    rec.vc_pos = sh.vc_pos;
    rec.given_len = sh.lens[0];
    rec.family_len = sh.lens[1];
    rec.dob_len = sh.lens[2];
    rec.nullifier_len = sh.null_len;
    for (int k = 0; k < 32; k++) rec.tbs_sha256[k] = sh.sha256[k];
    for (int k = 0; k < 64; k++) rec.nullifier_sha512[k] = sh.sha512[k];
    for (int k = 0; k < 64; k++) rec.nullifier[k] = sh.nullifier[k];
    for (int k = 0; k < 3; k++) store_fr_le(rec.pub[k], out[k]);
    if (witness) {  // witness[1..3] = out[0..2] (circom puts main's outputs first)
      uint8_t* wp = witness + (size_t)pass * wit_stride;
      for (int k = 0; k < 3; k++) store_fr_le(wp + 32 * (1 + k), out[k]);
    }
  }
  if (records) records[pass] = rec;
}

void check_params(const nzcb_nzcp_params* p) {
  if (!p) throw Error(NZCB_ERR_ARG, "nzcp: params is NULL");
  if (p->max_tbs_bytes < 1 || p->max_tbs_bytes > kMaxBytes)
    throw Error(NZCB_ERR_ARG, "nzcp: MaxToBeSignedBytes must be in [1, 512] (Sha256Var(3) holds 4096 bits)");
  if (p->max_array_len_vc < 0 || p->max_array_len_vc > kMaxArray)
    throw Error(NZCB_ERR_ARG, "nzcp: MaxCborArrayLenVC must be in [0, 8]");
  if (p->max_map_len_vc < 0 || p->max_map_len_vc > kMaxMap)
    throw Error(NZCB_ERR_ARG, "nzcp: MaxCborMapLenVC must be in [0, 32]");
}

}  // namespace nzcp
}  // namespace nzcb

using namespace nzcb;

extern "C" {

size_t nzcb_nzcp_input_signals(const nzcb_nzcp_params* prm) {
  if (!prm || prm->max_tbs_bytes < 1) return 0;
  return (size_t)prm->max_tbs_bytes * 8 + 1 + nzcp::kData;
}

int nzcb_nzcp_witness_dev(int device, const nzcb_nzcp_params* prm, const void* dev_inputs, int count,
                          void* dev_records, void* dev_witness, size_t witness_stride, void* stream, nzcb_err* err) {
  try {
    nzcp::check_params(prm);
    if (count < 0 || (count > 0 && !dev_inputs)) throw Error(NZCB_ERR_ARG, "nzcp: bad inputs");
    if (dev_witness && witness_stride < 4 * 32) throw Error(NZCB_ERR_ARG, "nzcp: witness stride < 4 signals");
    if (count == 0) return NZCB_OK;
    NZ_HIP(hipSetDevice(device));
    hipLaunchKernelGGL(nzcp::nzcp_witness_kernel, dim3(count), dim3(nzcp::kThreads), 0, (hipStream_t)stream,
                       (const uint8_t*)dev_inputs, count, *prm, (nzcb_nzcp_record*)dev_records,
                       (uint8_t*)dev_witness, witness_stride);
    NZ_HIP(hipGetLastError());
    return NZCB_OK;
  } catch (const Error& e) {
    set_err(err, e.code, e.what());
    return e.code;
  } catch (const std::exception& e) {
    set_err(err, NZCB_ERR_INTERNAL, e.what());
    return NZCB_ERR_INTERNAL;
  }
}

int nzcb_nzcp_witness(int device, const nzcb_nzcp_params* prm, const uint8_t* inputs, int count,
                      nzcb_nzcp_record* records, nzcb_err* err) {
  try {
    nzcp::check_params(prm);
    if (count < 0 || (count > 0 && (!inputs || !records))) throw Error(NZCB_ERR_ARG, "nzcp: bad buffers");
    if (count == 0) return NZCB_OK;
    NZ_HIP(hipSetDevice(device));
    size_t in_bytes = nzcb_nzcp_input_signals(prm) * 32 * (size_t)count;
    DevBuf<uint8_t> din(in_bytes);
    DevBuf<nzcb_nzcp_record> drec((size_t)count);
    NZ_HIP(hipMemcpy(din.p, inputs, in_bytes, hipMemcpyHostToDevice));
    int rc = nzcb_nzcp_witness_dev(device, prm, din.p, count, drec.p, nullptr, 0, nullptr, err);
    if (rc) return rc;
    NZ_HIP(hipMemcpy(records, drec.p, drec.bytes(), hipMemcpyDeviceToHost));
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
