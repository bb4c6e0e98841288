// PLONK prover rounds 1-5 on gfx950 (snarkjs 0.4.12 plonk_prove restated).
//
// Reference: snarkjs@0.4.12 src/plonk_prove.js [EXT] (/root/reference/yarn.lock:7279-7292),
// called by the reference's dapp / CLI on the zkey built at /root/reference/Makefile:59-62.
// Row-by-row spec: SURVEY.md §8a a3-a12. Every value below is a unique field or
// affine-curve element, so with the same blinding scalars the proof bytes are the
// ones snarkjs would print (parity pinned here against oracle/plonk.py).
//
// Design: the zkey is uploaded once (HBM-resident, LEM bytes as in the file) and
// every per-proof array stays on the device; the host only runs the Fiat-Shamir
// transcript (keccak over ~1 KB), the per-MSM window fold and a handful of Fr
// scalars. All data is kept in Montgomery form; MSM digit extraction converts.
// Sequential JS loops of the reference become parallel scans:
//   * Z grand product  -> chunked batch inversion + exclusive prefix-product scan
//   * divPol1          -> suffix linear-recurrence scan y_i = x_i + d*y_{i+1}
//   * evalPol (Horner) -> chunked Horner * x^(chunk start) + tree sum
#include <rocprofiler-sdk-roctx/roctx.h>
#include "lagrange.h"
#include "prover.h"
#include "transcript.h"

#include <cstring>
#include <cerrno>
#include <string>
#include <sys/random.h>

#include "keccak.h"

namespace nzcb {

static constexpr int kT = 256;
static constexpr uint32_t kZeroRef = 0xffffffffu;

// ----------------------------------------------------------------------------
// kernels
// ----------------------------------------------------------------------------
__global__ void k_wit_to_mont(const Fr* __restrict__ in, Fr* __restrict__ out, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = (i == 0) ? Fr::zero() : to_mont(in[i]);  // "First element in plonk is not used"
}

__global__ void k_additions(const AddRec* __restrict__ recs, uint32_t count, Fr* __restrict__ wit) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const AddRec r = recs[i];
  Fr a = r.ai == kZeroRef ? Fr::zero() : wit[r.ai];
  Fr b = r.bi == kZeroRef ? Fr::zero() : wit[r.bi];
  wit[r.dst] = r.ac * a + r.bc * b;
}

// Host writes of small results (the prover's mailbox, coherent pinned memory): common.h host_put

__global__ void k_build_abc(const uint32_t* __restrict__ am, const uint32_t* __restrict__ bm,
                            const uint32_t* __restrict__ cm, uint32_t nc, uint32_t n, const Fr* __restrict__ wit,
                            uint32_t nvars, Fr* __restrict__ A, Fr* __restrict__ B, Fr* __restrict__ C,
                            uint32_t npub, Fr* __restrict__ mb_apub, Fr* __restrict__ mb_pubw) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < npub) {  // the public signals witness[1..nPublic] into the mailbox (Prover::prove's output)
    host_put(mb_pubw + i, 1 + i < nvars ? wit[1 + i] : Fr::zero());
  }
  if (i >= n) {
    if (i < npub) host_put_done();
    return;
  }
  Fr a = Fr::zero(), b = Fr::zero(), c = Fr::zero();
  if (i < nc) {
    uint32_t ia = am[i], ib = bm[i], ic = cm[i];
    if (ia < nvars) a = wit[ia];
    if (ib < nvars) b = wit[ib];
    if (ic < nvars) c = wit[ic];
  }
  A[i] = a;
  B[i] = b;
  C[i] = c;
  if (i < npub) {  // A's public-gate values: the beta transcript's public inputs (round 2)
    host_put(mb_apub + i, a);
    host_put_done();
  }
}

// round 3's host inputs in one dispatch: the top coefficients of A, B, C (n-4 .. n+1) and Z
// (n-3 .. n+2) and the flags word, into the mailbox (five copies until round 6)
__global__ void k_tops(const Fr* __restrict__ pa, const Fr* __restrict__ pb, const Fr* __restrict__ pc,
                       const Fr* __restrict__ pz, size_t n, const uint32_t* __restrict__ flags, Fr* __restrict__ mb) {
  const int t = threadIdx.x;  // 32 threads
  if (t < 24) {
    const int k = t / 6, j = t % 6;
    const Fr* src = k == 0 ? pa + (n - 4) : k == 1 ? pb + (n - 4) : k == 2 ? pc + (n - 4) : pz + (n - 3);
    host_put(mb + t, src[j]);
  } else if (t == 24) {
    Fr f = Fr::zero();
    f.v[0] = *flags;
    host_put(mb + 24, f);
  }
  host_put_done();
}

struct BlindIdx {
  int idx[3];
  int count;
};

// p1 = p + (sum_k pz_k X^k)(X^n - 1): pol[n+k] = pz_k, pol[k] -= pz_k  (to4T)
__global__ void k_blind(Fr* pol, size_t n, const Fr* __restrict__ bl, BlindIdx bi) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (int k = 0; k < bi.count; k++) {
    Fr b = bl[bi.idx[k]];
    pol[n + k] = b;
    pol[k] = pol[k] - b;
  }
}

// A, B, C committed in the Lagrange basis (Prover::ltau): their blinding scalars follow
// the n evaluations, matching ltau[n] = [tau^n] - [1] and ltau[n+1] = [tau^(n+1)] - [tau]
// (k_blind's b_lo + b_hi X times X^n - 1)
__global__ void k_abc_tail(Fr* A, Fr* B, Fr* C, size_t n, const Fr* __restrict__ bl) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  A[n] = bl[2];
  A[n + 1] = bl[1];
  B[n] = bl[4];
  B[n + 1] = bl[3];
  C[n] = bl[6];
  C[n + 1] = bl[5];
}

// A, B, C in one MSM schedule (round 6); NZCB_ABC_SETS=0 commits them as three MSMs
static bool abc_sets_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("NZCB_ABC_SETS");
    return !e || std::atoi(e) != 0;
  }();
  return v;
}

static bool lagrange_commit_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("NZCB_LAGRANGE_COMMIT");
    return !e || std::atoi(e) != 0;
  }();
  return v;
}

// w4^i from two small tables (4n-th roots of unity)
__device__ __forceinline__ Fr root4(const Fr* __restrict__ lo, const Fr* __restrict__ hi, size_t i) {
  return lo[i & 4095] * hi[i >> 12];
}

struct PermArgs {
  F29 beta, beta_s;                      // Shoup pair of beta (mul_shoup: w, floor(w 2^261 / r))
  F29 k1beta, k1beta_s, k2beta, k2beta_s;  // ... of k1 beta, k2 beta (read only when k23 == 0)
  F29 gamma256;                          // gamma at exponent 256 (its Montgomery-256 form)
  int k23;                               // k1 = 2, k2 = 3 (snarkjs getK1K2 for BN254): k beta w by additions
};
// Shoup pair (w, ws) of a Montgomery-256 constant c: w = c's canonical value, ws = floor(w
// 2^261 / r) from m = w 2^261 mod r = c 2^5 mod r (as ntt.hip's ntt_tw29_kernel; host)
static void shoup_pair(const Fr& c, F29& w, F29& ws) {
  Fr m = c;
  for (int k = 0; k < 5; k++) m = m + m;
  w = split29(from_mont(c));
  ws = mul_lo261(split29(m), f29_const(Fr29::NINV));
}

// c * 2^5 split into the 9x29 radix: the Montgomery-261 operand of mul_fr29 for a
// Montgomery-256 constant c
static F29 fr29_operand(Fr c) {
  for (int k = 0; k < 5; k++) c = c + c;
  return split29(c);
}

// ---- coalesced tile scans (round 2's grand product, round 5's divPol1) --------------
// A workgroup owns a tile of kTileN consecutive elements and thread t the kPer consecutive
// elements [kPer t, kPer t + kPer) of it, so the sequential part of a scan runs in
// registers. Loads and stores go through LDS: coalesced (consecutive lanes, consecutive
// 32-byte elements) on the HBM side, and with one word of padding per 4 elements (word
// 8 e + e / 4 + w) both the coalesced pass and the per-thread pass hit 32 distinct banks per
// 32-lane half for kPer = 2 and 4 (ds_read_b32 / ds_write_b32 bank by (a / 4) mod 32).
// The chunk-per-thread scans these replace (32 elements per thread read
// straight from HBM, 1 KB apart per lane) ran at 0.06-0.3 of the HBM rate.
// kPer = 4 (175 VGPRs, no scratch, 2 waves per SIMD) against 2 (132 VGPRs, 48 B of scratch
// in k_perm_tile): bench +0.9 % on one box (profiles/r4_window_ab.txt); -DNZ_KPER=2 for A/B
#ifndef NZ_KPER
#define NZ_KPER 4
#endif
static constexpr int kPer = NZ_KPER;  // elements per thread in the tile scans
static constexpr int kTileN = kT * kPer;                // 1024
static constexpr int kStageWords = kTileN * 8 + kTileN / 4;

__device__ __forceinline__ int stage_word(int e) { return e * 8 + e / 4; }

// elements [base, base + kTileN) of f(g) (g < len; zero past it) -> use(j, x) for this
// thread's kPer elements j (consumed as they leave LDS: no array of them stays live)
template <class F, class U>
__device__ __forceinline__ void stage_use(F&& f, size_t base, size_t len, uint32_t* lds, U&& use) {
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    const int e = k * kT + (int)threadIdx.x;
    const size_t g = base + (size_t)e;
    const Fr v = g < len ? f(g) : Fr::zero();
#pragma unroll
    for (int w = 0; w < 8; w++) lds[stage_word(e) + w] = v.v[w];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kPer; j++) {
    const int e = kPer * (int)threadIdx.x + j;
    Fr x;
#pragma unroll
    for (int w = 0; w < 8; w++) x.v[w] = lds[stage_word(e) + w];
    use(j, x);
  }
  __syncthreads();
}
template <class F>
__device__ __forceinline__ void stage_in(F&& f, size_t base, size_t len, uint32_t* lds, Fr (&out)[kPer]) {
  stage_use(f, base, len, lds, [&](int j, const Fr& x) { out[j] = x; });
}

// this thread's kPer elements -> dst[base + e] for base + e < len (coalesced)
__device__ __forceinline__ void stage_out(const Fr (&v)[kPer], size_t base, size_t len, uint32_t* lds, Fr* dst) {
#pragma unroll
  for (int j = 0; j < kPer; j++) {
    const int e = kPer * (int)threadIdx.x + j;
#pragma unroll
    for (int w = 0; w < 8; w++) lds[stage_word(e) + w] = v[j].v[w];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    const int e = k * kT + (int)threadIdx.x;
    const size_t g = base + (size_t)e;
    Fr x;
#pragma unroll
    for (int w = 0; w < 8; w++) x.v[w] = lds[stage_word(e) + w];
    if (g < len) dst[g] = x;
  }
  __syncthreads();
}

// Workgroup scans (exclusive, over the kT threads in thread order) in two levels: a
// Kogge-Stone over each wave's 64 lanes by shuffles (no barrier), then the kT / 64 wave
// totals through LDS (one barrier pair). Round 3's form, a Kogge-Stone over all kT threads in
// LDS, paid two barriers per step (32 per product scan pair of k_perm_tile).
__device__ __forceinline__ Fr shfl_fr(const Fr& v, int src) {
  Fr o;
#pragma unroll
  for (int w = 0; w < 8; w++) o.v[w] = __shfl(v.v[w], src, 64);
  return o;
}
__device__ __forceinline__ F29 shfl_fr(const F29& v, int src) {
  F29 o;
#pragma unroll
  for (int w = 0; w < 9; w++) o.v[w] = __shfl(v.v[w], src, 64);
  return o;
}
struct MulOp {
  using T = Fr;
  static constexpr bool kCheap = false;
  __device__ Fr operator()(const Fr& a, const Fr& b) const { return a * b; }
  __device__ static Fr id() { return Fr::one(); }
};
struct AddOp {
  using T = Fr;
  static constexpr bool kCheap = true;
  __device__ Fr operator()(const Fr& a, const Fr& b) const { return a + b; }
  __device__ static Fr id() { return Fr::zero(); }
};
// products of Montgomery-261 values in the 9x29 radix (F29 of v 2^261 mod r, the one
// exponent that a product of any number of factors keeps: mul29 takes 2^261 off)
struct Mul29Op {
  using T = F29;
  static constexpr bool kCheap = false;
  __device__ F29 operator()(const F29& a, const F29& b) const { return mul29<Fr29>(a, b); }
  __device__ static F29 id() { return f29_const(Fr29::ONE); }
};
// kSuffix = false: op of v_t' over t' < t; true: over t' > t, for the NT threads of the
// workgroup. sh: >= NT / 64 entries. *total (when given) = op over all NT values, valid in
// thread 0. Up to 4 waves an addition scan combines the wave totals directly (wave-uniform
// branches: wave w applies w of them, thread 0 all for the total); a product scan, and any
// scan past 4 waves, has the first wave scan them by shuffles and every wave apply one
// (k_perm_tile's two scans: 12 instead of 15 wave-products per workgroup).
template <bool kSuffix, class Op, int NT = kT>
__device__ __forceinline__ typename Op::T block_scan_excl(const typename Op::T& v, typename Op::T* sh,
                                                          typename Op::T* total) {
  using T = typename Op::T;
  constexpr int NW = NT / 64;
  static_assert(NW >= 1 && NW <= 64 && NT % 64 == 0, "whole waves, at most 64");
  const Op op;
  const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
  T inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int src = kSuffix ? lane + d : lane - d;
    const T o = shfl_fr(inc, src & 63);
    if (kSuffix ? lane + d < 64 : lane >= d) inc = op(inc, o);
  }
  T ex = shfl_fr(inc, (kSuffix ? lane + 1 : lane - 1) & 63);
  if (kSuffix ? lane == 63 : lane == 0) ex = Op::id();
  if (kSuffix ? lane == 0 : lane == 63) sh[wv] = inc;  // the wave's total
  __syncthreads();
  if constexpr (NW <= 4 && Op::kCheap) {
#pragma unroll
    for (int k = 0; k < NW; k++)  // wave-uniform: the other waves' totals on this side
      if (kSuffix ? k > wv : k < wv) ex = op(ex, sh[k]);
    if (total && threadIdx.x == 0) {
      T t = sh[0];
#pragma unroll
      for (int k = 1; k < NW; k++) t = op(t, sh[k]);
      *total = t;
    }
    __syncthreads();
  } else {
    T tot_all = Op::id();
    if (wv == 0) {  // exclusive scan of the NW wave totals in lanes < NW, back into sh
      T w = lane < NW ? sh[lane] : Op::id();
#pragma unroll
      for (int d = 1; d < NW; d <<= 1) {
        const int src = kSuffix ? lane + d : lane - d;
        const T o = shfl_fr(w, src & 63);
        if (kSuffix ? lane + d < NW : (lane >= d && lane < NW)) w = op(w, o);
      }
      T wex = shfl_fr(w, (kSuffix ? lane + 1 : lane - 1) & 63);
      if (kSuffix ? lane == NW - 1 : lane == 0) wex = Op::id();
      tot_all = shfl_fr(w, kSuffix ? 0 : NW - 1);
      if (lane < NW) sh[lane] = wex;  // no other wave reads sh before the barrier below
    }
    __syncthreads();
    ex = op(ex, sh[wv]);
    if (total && threadIdx.x == 0) *total = tot_all;
    __syncthreads();
  }
  return ex;
}
__device__ __forceinline__ Fr block_prod_excl(const Fr& v, Fr* sh, Fr& total) {
  return block_scan_excl<false, MulOp>(v, sh, &total);
}
__device__ __forceinline__ Fr block_prod_excl_suffix(const Fr& v, Fr* sh) {
  return block_scan_excl<true, MulOp>(v, sh, nullptr);
}
__device__ __forceinline__ Fr block_sum_excl_suffix(const Fr& v, Fr* sh, Fr& total) {
  return block_scan_excl<true, AddOp>(v, sh, &total);
}

// Round 2 without a single inversion per element or per workgroup:
//   Z_i = prod_{k<i} num_k / den_k = (prod_{k<i} num_k) (prod_{k>=i} den_k) / prod_k den_k,
// with num_i = (a + b w^i + g)(b + k1 b w^i + g)(c + k2 b w^i + g) and
//      den_i = (a + b s1_i + g)(b + b s2_i + g)(c + b s3_i + g):
// an exclusive prefix product of the numerators, an inclusive suffix product of the
// denominators and ONE inversion per proof (of prod den, which the copy-constraint check
// compares with prod num anyway). A workgroup computes its tile's num / den, the tile-local
// scans (thread-local over kPer elements, Kogge-Stone over the threads) and writes
// Zloc_i = Nloc_excl_i * Dloc_suffix_i and the tile totals; k_perm_factors and
// k_apply_tiles multiply in the other tiles' totals and the inverse. The sigma evaluations
// come from contiguous copies (Prover::sig_h), not at stride 4 from the 4n evaluations.
// Round 3 ran a batch inversion per 32-element chunk per thread (1.24 ms at 2^21, the
// chunks 1 KB apart per lane, den / prefix arrays written and read back through HBM).
#ifndef NZ_PERM_WAVES
// waves per SIMD the grand-product tile kernel is compiled for: at 2 it takes 247 VGPRs and
// no scratch; the exponent-261 form before it took 223 at 2 and spilled 188 B at 3 (168
// VGPRs): 394 against 404 us per launch in a single-lane proof, same bench
// (profiles/r5_perm_waves_ab.txt)
#define NZ_PERM_WAVES 2
#endif
// Every product runs in the 9x29 radix (round 5; until round 4 the factors' products and both
// scans were 8x32 products, 13 of them per element). The factors stay at exponent 256: x is
// the witness value's Montgomery-256 form as it is, b s_k and k b w^i are Shoup products of
// the Montgomery-256 sigma / w^i (table w_h) by the canonical beta, k beta, and gamma is
// Montgomery-256. Each real element's num and den then carry the same 2^-15 against their
// exponent-261 values (three factors at 256, two Montgomery products), and every quantity
// the proof reads is a ratio with as many num as den factors: a local Z_i holds the tile's
// num_k (k < i) and den_k (k >= i), one each per real element, its F_T the other tiles'
// totals, and 1 / prod den the rest (prod num = prod den, the copy-constraint check, holds
// with both sides scaled alike). Past n the factors are the exponent-261 one. Against the
// exponent-261 factors (fr_to261 shifts, Montgomery products by beta 2^266) this drops three
// limb shifts and four products' 28 reduction instructions each (Shoup), and the factors of
// the k >= 1 columns feed their product unnormalized against the normalized num / den. Their
// limbs: x + 2 b w + g < 4 2^29 (f29.h's one factor < 2^31), x + 3 b w + g < 5 2^29, one step
// past it: a column of that product is <= 9 (5 2^29 2^29 + 2^58) + 2^35 < 2^63.8 < 2^64.
__device__ __forceinline__ F29 add3_nn29(const F29& a, const F29& b, const F29& c) {  // unnormalized
  F29 r;
#pragma unroll
  for (int l = 0; l < 9; l++) r.v[l] = a.v[l] + b.v[l] + c.v[l];
  return r;
}
__global__ void __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(NZ_PERM_WAVES, 8)))
k_perm_tile(const Fr* __restrict__ A, const Fr* __restrict__ B, const Fr* __restrict__ C,
            const Fr* __restrict__ sig_h, size_t n, const Fr* __restrict__ w_h, PermArgs pa, Fr* __restrict__ Z,
            Fr* __restrict__ ntot, Fr* __restrict__ dtot) {
  __shared__ uint32_t stg[kStageWords];
  __shared__ F29 sh[kT / 64];  // the scans' wave totals
  const int tid = threadIdx.x;
  const size_t base = (size_t)blockIdx.x * kTileN;
  const size_t e0 = base + (size_t)kPer * tid;
  const F29 beta = pa.beta, beta_s = pa.beta_s, gamma = pa.gamma256;  // no byval copy in scratch
  const bool k23 = pa.k23 != 0;
  F29 num[kPer], den[kPer], bw[kPer], bs[kPer];
#pragma unroll 1
  for (int k = 0; k < 3; k++) {
    // sigma_k first: bs = b s_k, for den *= x + b s_k + g below
    stage_use([&](size_t g) { return sig_h[(size_t)k * n + g]; }, base, n, stg,
              [&](int j, const Fr& x) { bs[j] = mul_shoup(split29(x), beta, beta_s); });
    // k b w: b w, 2 b w, 3 b w when k1, k2 = 2, 3, what snarkjs getK1K2 finds for BN254 (bw[]
    // keeps b w^i), else one Shoup product per column
    if (k == 0 || !k23) {
      const F29 kb = k == 0 ? beta : (k == 1 ? pa.k1beta : pa.k2beta);
      const F29 kbs = k == 0 ? beta_s : (k == 1 ? pa.k1beta_s : pa.k2beta_s);
#pragma unroll
      for (int j = 0; j < kPer; j++) bw[j] = mul_shoup(split29(e0 + j < n ? w_h[e0 + j] : Fr::zero()), kb, kbs);
    }
    // witness column: num *= x + k b w + g, den *= x + b s_k + g
    const Fr* col = k == 0 ? A : B;
    if (k == 2) col = C;
    stage_use([&](size_t g) { return col[g]; }, base, n, stg,
              [&](int j, const Fr& x) {
                F29 kbw = bw[j];  // < 3 r
                if (k23 && k == 1) {  // 2 b w, 3 b w unnormalized: f's limbs < 4 2^29, 5 2^29 (below)
#pragma unroll
                  for (int l = 0; l < 9; l++) kbw.v[l] = bw[j].v[l] << 1;
                } else if (k23 && k == 2) {
#pragma unroll
                  for (int l = 0; l < 9; l++) kbw.v[l] = (bw[j].v[l] << 1) + bw[j].v[l];
                }
                const F29 xs = split29(x);
                if (k == 0) {
                  num[j] = add3_29(xs, kbw, gamma);   // < 5 r, normalized (k >= 1: < 11 r)
                  den[j] = add3_29(xs, bs[j], gamma);  // < 5 r
                } else {
                  num[j] = mul29<Fr29>(num[j], add3_nn29(xs, kbw, gamma));
                  den[j] = mul29<Fr29>(den[j], add3_nn29(xs, bs[j], gamma));
                }
              });
  }
  const F29 one = f29_const(Fr29::ONE);
#pragma unroll
  for (int j = 0; j < kPer; j++)  // past n: factor 1
    if (e0 + j >= n) num[j] = den[j] = one;
  // thread-local: the product of num, bs = inclusive suffix of den; after the scans the
  // prefix of num restarts from c, so each output is one product (15 products per thread
  // against 17 with a stored prefix times c)
  F29 ntl = num[0];
#pragma unroll
  for (int j = 1; j < kPer; j++) ntl = mul29<Fr29>(ntl, num[j]);
  bs[kPer - 1] = den[kPer - 1];
#pragma unroll
  for (int j = kPer - 2; j >= 0; j--) bs[j] = mul29<Fr29>(bs[j + 1], den[j]);
  F29 nt;
  const F29 np = block_scan_excl<false, Mul29Op>(ntl, sh, &nt);
  const F29 ds = block_scan_excl<true, Mul29Op>(bs[0], sh, nullptr);
  // c at exponent 256: the last product of each element lands in Montgomery-256
  F29 pre = mul29<Fr29>(mul29<Fr29>(np, ds), f29_const(Fr29::C256));
  Fr out[kPer];
#pragma unroll
  for (int j = 0; j < kPer; j++) {
    out[j] = join_fr29(mul29<Fr29>(pre, bs[j]));
    if (j + 1 < kPer) pre = mul29<Fr29>(pre, num[j]);
  }
  stage_out(out, base, n, stg, Z);
  if (tid == 0) {
    ntot[blockIdx.x] = fr_from261(nt);
    dtot[blockIdx.x] = fr_from261(mul29<Fr29>(ds, bs[0]));  // thread 0: its own suffix times the others'
  }
}

// F_T = (prod_{T'<T} N_T') (prod_{T'>T} D_T') (one workgroup; each thread a run of
// consecutive tiles); totals[0] = prod N, totals[1] = prod D (round 2's copy-constraint check).
// 1 / prod D is the host's (Prover::prove reads the totals for the check anyway): a
// single-lane Fermat inversion here was most of this kernel's 0.6 ms.
__global__ void __launch_bounds__(1024)
k_perm_factors(const Fr* __restrict__ ntot, const Fr* __restrict__ dtot, int ntiles, Fr* __restrict__ F,
               Fr* __restrict__ totals) {  // totals: the mailbox (host memory)
  __shared__ Fr sh[1024 / 64];  // the scans' wave totals
  const int tid = threadIdx.x;
  const int per = (ntiles + 1023) / 1024;
  const int t0 = min(tid * per, ntiles), t1 = min(t0 + per, ntiles);
  Fr pn = Fr::one(), pd = Fr::one();
  for (int t = t0; t < t1; t++) {
    pn = pn * ntot[t];
    pd = pd * dtot[t];
  }
  // exclusive prefix of pn, exclusive suffix of pd over the 1024 threads
  Fr nall, dall;
  const Fr npre = block_scan_excl<false, MulOp, 1024>(pn, sh, &nall);
  const Fr dsuf = block_scan_excl<true, MulOp, 1024>(pd, sh, &dall);
  if (tid == 0) {
    host_put(totals, nall);
    host_put(totals + 1, dall);
    host_put_done();
  }
  // within the run: prefix of N (forward), suffix of D (backward)
  Fr run = npre;
  for (int t = t0; t < t1; t++) {
    F[t] = run;
    run = run * ntot[t];
  }
  Fr sd = dsuf;
  for (int t = t1 - 1; t >= t0; t--) {
    F[t] = F[t] * sd;
    sd = sd * dtot[t];
  }
}

// Z[i] *= F[i / kTileN] / prod D (coalesced): one workgroup per tile, F_T / prod D once per
// thread for its kPer elements (1 + 1 / kPer products per element instead of 2)
__global__ void __launch_bounds__(kT)
k_apply_tiles(Fr* __restrict__ x, size_t m, const Fr* __restrict__ F, Fr inv_d) {
  const Fr f = F[blockIdx.x] * inv_d;
  const size_t base = (size_t)blockIdx.x * kTileN + threadIdx.x;
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    const size_t i = base + (size_t)k * kT;
    if (i < m) x[i] = x[i] * f;
  }
}

// Round 5's divPol1: y_i = x_i + d y_{i+1} over i < m, x_i =
// src[i + 1] (x_{m-1} = 0), y_m = 0, by tiles. Each thread runs the recurrence over its
// kPer elements (head h_t = sum_j x_(kPer t + j) d^j). Across the threads the recurrence is
// a weighted suffix sum: the true y at thread t's first element is
//   Y_t = d^(-kPer t) (sum_(t' >= t) h_t' d^(kPer t') + c d^kTileN)
// with c the tile's carry-in (the true y at the next tile's first element), so with the
// tables P[t] = d^(kPer t), Pinv[t] = d^(-kPer t) (LinTab, built on the host once per d)
// the scan is of additions: two products per thread instead of two per Kogge-Stone step
// (round 3's multiplicative scan, 16 products per thread). Two passes: kWrite = false writes
// the tile heads (c = 0), which a small scan turns into the true carries; kWrite = true
// recomputes the tile with its carry and writes y. d = 0 (y = x) works with Pinv = 0.
struct LinTab {
  Fr P[kT + 1];     // d^(kPer t)
  Fr Pinv[kT + 1];  // d^(-kPer t) (0 for t > 0 when d = 0)
  Fr dp[kPer + 1];  // d^j
};
// ... and per tile T (Prover::lin_tables, after the LinTab): Q[T] = D^T, Qinv[T] = D^(-T) with
// D = d^kTileN, so the tile heads h_T chain the same way: H_T = Qinv[T] sum_(T' >= T) h_T' Q[T']
static_assert(sizeof(LinTab) % sizeof(Fr) == 0, "LinTab is stored as Fr words");

template <bool kWrite>
__global__ void __launch_bounds__(kT)
k_lin_tile(const Fr* __restrict__ src, size_t m, const LinTab* __restrict__ tab, const Fr* __restrict__ carry,
           Fr* __restrict__ out) {
  __shared__ uint32_t stg[kStageWords];
  __shared__ Fr sh[kT / 64];  // the scan's wave totals
  const int tid = threadIdx.x;
  const size_t base = (size_t)blockIdx.x * kTileN;
  Fr x[kPer];
  stage_in([&](size_t g) { return src[g + 1]; }, base, m - 1, stg, x);
  const Fr d = tab->dp[1];
  Fr y = Fr::zero();
#pragma unroll
  for (int j = kPer - 1; j >= 0; j--) {
    y = x[j] + d * y;
    x[j] = y;
  }
  Fr total;
  Fr ex = block_sum_excl_suffix(y * tab->P[tid], sh, total);
  if (!kWrite) {
    if (tid == 0) out[blockIdx.x] = total;  // h_T
    return;
  }
  if (carry) ex = ex + carry[blockIdx.x + 1] * tab->P[kT];
  const Fr next = ex * tab->Pinv[tid + 1];  // the true y at element kPer (t + 1) of the tile
#pragma unroll
  for (int j = 0; j < kPer; j++) x[j] = x[j] + tab->dp[kPer - j] * next;
  stage_out(x, base, m, stg, out);
}

// Q[T] = D^T and Qinv[T] = Di^T for T < count (square-and-multiply per thread)
__global__ void k_pow_tiles(Fr D, Fr Di, int count, Fr* __restrict__ Q, Fr* __restrict__ Qinv) {
  const int T = blockIdx.x * blockDim.x + threadIdx.x;
  if (T >= count) return;
  Fr a = Fr::one(), b = Fr::one(), pa = D, pb = Di;
  for (int e = T; e; e >>= 1) {
    if (e & 1) {
      a = a * pa;
      b = b * pb;
    }
    pa = sqr(pa);
    pb = sqr(pb);
  }
  Q[T] = a;
  Qinv[T] = b;
}

// the true tile heads from the tile-local ones: H_T = Qinv[T] sum_(T' >= T) h_T' Q[T'] for
// T < m, H_m = 0 (one workgroup: each thread a run of tiles, then a suffix sum of additions
// over the threads); h[T] is replaced by H_T
__global__ void __launch_bounds__(1024) k_tile_heads(Fr* __restrict__ h, int m, const Fr* __restrict__ Q,
                                                     const Fr* __restrict__ Qinv) {
  __shared__ Fr sh[1024 / 64];  // the scan's wave totals
  const int tid = threadIdx.x;
  const int per = (m + 1023) / 1024;
  const int t0 = min(tid * per, m), t1 = min(t0 + per, m);
  Fr run = Fr::zero();
  for (int T = t0; T < t1; T++) run = run + h[T] * Q[T];
  // exclusive suffix sum of the runs over the threads
  Fr suf = block_scan_excl<true, AddOp, 1024>(run, sh, nullptr);
  for (int T = t1 - 1; T >= t0; T--) {
    suf = suf + h[T] * Q[T];
    h[T] = suf * Qinv[T];
  }
  if (tid == 0) h[m] = Fr::zero();
}

// contiguous sigma_k(w^i) = the 4n evaluation at 4 i (once per context)
__global__ void k_stride4(const Fr* __restrict__ src, size_t n, Fr* __restrict__ dst) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[4 * i];
}

struct QArgs {
  Fr beta, gamma, alpha, alpha2, bk1, bk2;  // bk1 = beta*k1, bk2 = beta*k2
  Fr zhinv[4];                              // 1 / Z_H(x_i), which depends on i mod 4 only
};

// Round 3, evaluated on the coset x_i = g * w4^i of the 4n
// domain, where Z_H(x_i) = g^n w4^(i n) - 1 never vanishes:
//   t(x_i) = [gate + alpha (perm_num - perm_den) + alpha^2 (z - 1) L1](x_i) / Z_H(x_i)
// with the blinded a, b, c, z evaluated directly. The quotient t (deg <= 3n+5 < 4n)
// is unique, so its coefficients equal snarkjs's T/Tz split over the plain 4n
// domain; this form needs ~25 Fr products per point instead of ~85, and a single
// 4n inverse NTT instead of two. z(w x_i) = z(x_{i+4}) since w = w4^4.
__global__ void __launch_bounds__(kT)
k_quotient_coset(const Fr* __restrict__ A, const Fr* __restrict__ B, const Fr* __restrict__ C,
                 const Fr* __restrict__ Z, const Fr* __restrict__ cq, const Fr* __restrict__ cs,
                 const Fr* __restrict__ cl, uint32_t npub, const Fr* __restrict__ Apub, size_t n,
                 const Fr* __restrict__ xlo, const Fr* __restrict__ xhi, QArgs q, Fr* __restrict__ T) {
  const size_t n4 = 4 * n;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const Fr a = A[i], b = B[i], c = C[i];
  const Fr x = xlo[i & 4095] * xhi[i >> 12];
  // gate: qm a b + ql a + qr b + qo c + qc + PI
  Fr gate = a * b * cq[i] + a * cq[n4 + i] + b * cq[2 * n4 + i] + c * cq[3 * n4 + i] + cq[4 * n4 + i];
  for (uint32_t j = 0; j < npub; j++) gate = gate - cl[j * n4 + i] * Apub[j];
  const Fr z = Z[i];
  const Fr bx = q.beta * x;
  Fr num = (a + bx + q.gamma) * (b + q.bk1 * x + q.gamma);
  num = num * (c + q.bk2 * x + q.gamma) * z;
  Fr den = (a + q.beta * cs[i] + q.gamma) * (b + q.beta * cs[n4 + i] + q.gamma);
  den = den * (c + q.beta * cs[2 * n4 + i] + q.gamma) * Z[(i + 4) & (n4 - 1)];
  const Fr e4 = (z - Fr::one()) * cl[i] * q.alpha2;
  T[i] = (gate + q.alpha * (num - den) + e4) * q.zhinv[i & 3];
}

// The same quotient in the 9x29-bit radix (f29.h, Fr29). Every summand is kept at the
// Montgomery exponent 2^256: a mul29 of exponents e1, e2 gives e1 + e2 - 261, so the
// per-context coset arrays are stored pre-scaled (qm * 2^10, ql / qr / qo / L_j * 2^5,
// x_lo * 2^5; kQ29Scale) and the scalars come in the exponent their product needs
// (QArgs29). Bounds: loaded values < r, products < 2r, mulsum29 of <= 4 terms < 2r,
// the final sum S < 9r < 2^257 (mul29's input limit), so T is canonical after one
// conditional subtraction. Used for nPublic <= 8 (two PI chunks at most).
constexpr uint32_t kQ29MaxPub = 8;

// the three-coset quotient (Prover::quot3, default; same box: bench 37.5 -> 38.9 proofs/s,
// profiles/r3_quot3_ab.txt); NZCB_QUOT3=0 restores the 4n coset (A/B runs)
static bool quot3_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("NZCB_QUOT3");
    return !(e && e[0] == '0');
  }();
  return on;
}
struct QArgs29 {
  F29 beta, bk1, bk2, alpha2, zhinv[4];  // exponent 261
  F29 gamma, negone;                     // exponent 256 (negone = r - 1)
  int k23;                               // k1 = 2, k2 = 3: k beta x as 2 beta x, 3 beta x
  F29 alpha;                             // exponent 276 (multiplies the exponent-241 permutation term)
};

template <int K>
__device__ __forceinline__ F29 q29_pi_chunk(const Fr* __restrict__ cl, const Fr* __restrict__ Apub, uint32_t j0,
                                            size_t n4, size_t i) {
  F29 pa[K], pb[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    pa[k] = split29(cl[(size_t)(j0 + k) * n4 + i]);  // L_j * 2^5
    pb[k] = split29(neg(Apub[j0 + k]));             // -Apub_j
  }
  return mulsum29<Fr29, K>(pa, pb);
}

__device__ __forceinline__ F29 q29_pi(const Fr* __restrict__ cl, const Fr* __restrict__ Apub, uint32_t j0,
                                      uint32_t cnt, size_t n4, size_t i) {
  switch (cnt) {
    case 1: return q29_pi_chunk<1>(cl, Apub, j0, n4, i);
    case 2: return q29_pi_chunk<2>(cl, Apub, j0, n4, i);
    case 3: return q29_pi_chunk<3>(cl, Apub, j0, n4, i);
    default: return q29_pi_chunk<4>(cl, Apub, j0, n4, i);
  }
}

// THREE (three-coset quotient): the points are c_j w^m, j < 3, stored coset-major at
// i = j n + m (x = g w4^(4m + j), Z(w x) at j n + (m + 1) mod n, 1/Z_H by j); otherwise
// the 4n coset g<w4> in natural order (x_i = g w4^i, Z(w x) at i + 4, 1/Z_H by i mod 4).
// Every array holds npts = 3n or 4n points per polynomial.
// 4 waves per SIMD (128 VGPRs, 24 B scratch) instead of the compiler's 3 (130 VGPRs):
// 1.084 -> 1.011 ms isolated, bench unchanged (profiles/r4_env_q4_ab.txt)
template <bool THREE>
__global__ void __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(4, 8)))
k_quotient_coset29(const Fr* __restrict__ A, const Fr* __restrict__ B, const Fr* __restrict__ C,
                   const Fr* __restrict__ Z, const Fr* __restrict__ cq, const Fr* __restrict__ cs,
                   const Fr* __restrict__ cl, uint32_t npub, const Fr* __restrict__ Apub, size_t n,
                   const Fr* __restrict__ xlo, const Fr* __restrict__ xhi, QArgs29 q, Fr* __restrict__ T) {
  const size_t n4 = (THREE ? 3 : 4) * n;  // points per array
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  size_t ix, izw;
  int cj;
  if (THREE) {
    const int lg = __ffsll((long long)n) - 1;
    const size_t j = i >> lg, m = i & (n - 1);
    ix = 4 * m + j;
    izw = j * n + ((m + 1) & (n - 1));
    cj = (int)j;
  } else {
    ix = i;
    izw = (i + 4) & (n4 - 1);
    cj = (int)(i & 3);
  }
  const F29 a = split29(A[i]), b = split29(B[i]), c = split29(C[i]), z = split29(Z[i]);
  // gate: qm a b + ql a + qr b + qo c + qc - sum_j L_j Apub_j
  F29 gate;
  {
    const F29 ga[4] = {mul29<Fr29>(a, b), a, b, c};
    const F29 gb[4] = {split29(cq[i]), split29(cq[n4 + i]), split29(cq[2 * n4 + i]), split29(cq[3 * n4 + i])};
    gate = add29(mulsum29<Fr29, 4>(ga, gb), split29(cq[4 * n4 + i]));  // < 3r
  }
  if (npub > 0) gate = add29(gate, q29_pi(cl, Apub, 0, npub < 4 ? npub : 4, n4, i));
  if (npub > 4) gate = add29(gate, q29_pi(cl, Apub, 4, npub - 4, n4, i));  // < 7r
  // permutation: (a + b x + g)(b + b k1 x + g)(c + b k2 x + g) z - (a + b s1 + g)(..)(..) z(w x)
  const F29 x = mul29<Fr29>(split29(xlo[ix & 4095]), split29(xhi[ix >> 12]));
  const F29 bx = mul29<Fr29>(q.beta, x);                   // < 2r
  const F29 bx2 = q.k23 ? add29(bx, bx) : mul29<Fr29>(q.bk1, x);  // < 4r
  const F29 bx3 = q.k23 ? add29(bx2, bx) : mul29<Fr29>(q.bk2, x);  // < 6r
  const F29 f1 = add29(add29(a, bx), q.gamma);   // < 4r
  const F29 f2 = add29(add29(b, bx2), q.gamma);  // < 6r
  const F29 f3 = add29(add29(c, bx3), q.gamma);  // < 8r < 2^257 (mul29's input limit)
  const F29 num = mul29<Fr29>(mul29<Fr29>(mul29<Fr29>(f1, f2), f3), z);  // exponent 241
  const F29 g1 = add29(add29(a, mul29<Fr29>(q.beta, split29(cs[i]))), q.gamma);
  const F29 g2 = add29(add29(b, mul29<Fr29>(q.beta, split29(cs[n4 + i]))), q.gamma);
  const F29 g3 = add29(add29(c, mul29<Fr29>(q.beta, split29(cs[2 * n4 + i]))), q.gamma);
  const F29 den = mul29<Fr29>(mul29<Fr29>(mul29<Fr29>(g1, g2), g3), split29(Z[izw]));
  // alpha (num - den) + alpha^2 (z - 1) L1, one reduction
  const F29 pa[2] = {q.alpha, q.alpha2};
  const F29 pb[2] = {sub29(num, den, Fr29::K2), mul29<Fr29>(add29(z, q.negone), split29(cl[i]))};
  const F29 S = add29(gate, mulsum29<Fr29, 2>(pa, pb));  // < 9r
  T[i] = join_fr29(mul29<Fr29>(S, q.zhinv[cj]));
}

// The three-coset quotient's divisibility check: N vanishes on H iff every gate holds
// there (the permutation part vanishes on H once round 2's copy check passed, z(1) = 1 by
// construction), i.e. qm a b + ql a + qr b + qo c + qc - PI = 0 at every w^m. The selectors
// on H are the zkey's 4n evaluations at stride 4, copied once per context into q_h
// (5 x n, contiguous: the stride-4 reads fetched a 128-byte line per 32-byte value)
__global__ void __launch_bounds__(kT)
k_gate_h(const Fr* __restrict__ A, const Fr* __restrict__ B, const Fr* __restrict__ C, const Fr* __restrict__ qh,
         size_t n, uint32_t npub, uint32_t* __restrict__ flags) {
  const size_t m = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  const Fr a = A[m], b = B[m], c = C[m];
  Fr g = qh[m] * a * b + qh[n + m] * a + qh[2 * n + m] * b + qh[3 * n + m] * c + qh[4 * n + m];
  if (m < npub) g = g - a;  // PI(w^m) = -pub_m, pub_m = A(w^m)
  if (!g.is_zero()) atomicOr(flags, 1u);
}

// t from its remainders v_j = (t mod (X^n - d_j)) / 4, j < 3, d_j = D w4^(j n) (w4^n = i,
// a 4th root of unity: d = D, iD, -D) and its top coefficients q3 = t[3n..3n+6):
// with w_j = v_j - d_j^3 q3 / 4 (c_j below), Q0 = w0 + w2 + 2 w1 - i (w0 - w2),
// Q1 = (w0 - w2) 2 / D, Q2 = (w0 + w2 - 2 w1 + i (w0 - w2)) / D^2; t = Q0 | Q1 | Q2 | q3
struct T3Args {
  Fr c0[6], c1[6], c2[6], q3[6];
  Fr i4, two_over_d, inv_d2;
};
__global__ void __launch_bounds__(kT)
k_t_combine(const Fr* __restrict__ V, size_t n, T3Args a, Fr* __restrict__ t) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  Fr v0 = V[k], v1 = V[n + k], v2 = V[2 * n + k];
  if (k < 6) {
    v0 = v0 - a.c0[k];
    v1 = v1 - a.c1[k];
    v2 = v2 - a.c2[k];
  }
  const Fr sm = v0 + v2, dl = v0 - v2, im = dl * a.i4, v12 = v1 + v1;
  t[k] = sm + v12 - im;
  t[n + k] = dl * a.two_over_d;
  t[2 * n + k] = (sm - v12 + im) * a.inv_d2;
  if (k < 6) t[3 * n + k] = a.q3[k];  // t has 3n + 6 coefficients (its buffer no more)
}

// w^i = w4^(4 i), i < n (Prover::w_h)
__global__ void k_root_n(Fr* __restrict__ out, const Fr* __restrict__ rlo, const Fr* __restrict__ rhi, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = root4(rlo, rhi, 4 * i);
}

// fault injection (nzcb_debug_inject_fault): one coefficient + 1
__global__ void k_fault_bump(Fr* x) {
  if (threadIdx.x == 0) x[0] = x[0] + Fr::one();
}

// x <- x * 2^e (mod r), canonical in and out: the exponent pre-scaling of kQ29
__global__ void k_dbl_pow(Fr* __restrict__ x, size_t m, int e) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  Fr v = x[i];
  for (int k = 0; k < e; k++) v = v + v;
  x[i] = v;
}

static F29 f29_exp(Fr v, int extra) {  // split29 of v * 2^extra (host)
  for (int k = 0; k < extra; k++) v = v + v;
  return split29(v);
}

// Round 4, all evaluations of one point set in two launches and one host round trip
// (eight separately synchronised Horner launches took 1.05 ms + 8 syncs per proof,
// profiles/r3_single_lane_phases.txt): k_eval_pows, k_eval_multi (one partial sum per
// workgroup and point, already times x^(4096 b)), k_eval_sum (the partial sums added).
static constexpr int kEvalMax = 8;
static constexpr int kEvalBits = 16;  // workgroup index bits (<= 2^16 workgroups of 4096 coefficients)
struct EvalSet {
  const Fr* p[kEvalMax];
  uint64_t len[kEvalMax];
  Fr x[kEvalMax];
  Fr x4096[kEvalMax];  // x^4096 (host), the base of the workgroup powers
  F29 x29[kEvalMax];  // x as the mul_fr29 operand
  F29 y29[kEvalMax];  // x^kT: the strided Horner's step (k_eval_multi)
  int np;
  int nbits;  // bits of the largest workgroup index
};

__device__ __forceinline__ F29 fr29_operand_dev(Fr c) {
#pragma unroll
  for (int k = 0; k < 5; k++) c = c + c;
  return split29(c);
}

// A workgroup evaluates the 4096 coefficients [4096 b, 4096 b + 4096) of each polynomial:
// thread t takes the coefficients 4096 b + t + 256 m (m < kEvalChunk2), so every load of a
// wave is 64 consecutive coefficients (round 3 gave each thread 16 consecutive ones, loads
// 512 B apart per lane), by Horner in y = x^256 over m; times x^t (k_eval_pows' table) the
// thread's terms carry their true power, and the workgroup adds them. NP evaluations side
// by side (independent chains).
static constexpr int kEvalChunk2 = 16;

// x_j^t for t < kT as mul_fr29 operands, and x_j^(4096 2^k) for k < nbits (pw2), one
// workgroup per evaluation point
__global__ void __launch_bounds__(kT) k_eval_pows(EvalSet es, F29* __restrict__ pw, Fr* __restrict__ pw2) {
  const int j = blockIdx.x, t = threadIdx.x;
  Fr a = Fr::one(), q = es.x[j];
  for (int e = t; e; e >>= 1) {
    if (e & 1) a = a * q;
    q = q * q;
  }
  pw[(size_t)j * kT + t] = fr29_operand_dev(a);
  if (t < es.nbits) {
    Fr z = es.x4096[j];
    for (int k = 0; k < t; k++) z = z * z;
    pw2[j * kEvalBits + t] = z;
  }
}

// sum of v over the workgroup's threads, in thread 0 (wave butterflies, then the wave totals)
__device__ __forceinline__ Fr block_sum_fr(const Fr& v, Fr* sh) {
  Fr x = v;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) x = x + shfl_fr(x, (int)(threadIdx.x & 63) ^ m);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = x;
  __syncthreads();
  Fr t = sh[0];
#pragma unroll
  for (int k = 1; k < kT / 64; k++) t = t + sh[k];
  __syncthreads();
  return t;
}

template <int NP>
__global__ void __launch_bounds__(kT) k_eval_multi(EvalSet es, const F29* __restrict__ pw, const Fr* __restrict__ pw2,
                                                   Fr* __restrict__ partial, int nblocks) {
  static_assert(NP <= kEvalMax && kEvalMax <= 4 * (kT / 64), "one 16-lane group per point");
  __shared__ Fr sh[kT / 64];
  __shared__ Fr bpow[kEvalMax];  // x_j^(4096 b): the product of pw2[j][k] over the set bits k of b
  __shared__ Fr bsum[kEvalMax];
  {
    const int l = (int)(threadIdx.x & 63), k = l & 15, j = 4 * (int)(threadIdx.x >> 6) + (l >> 4);
    Fr f = Fr::one();
    if (j < NP && k < es.nbits && ((blockIdx.x >> k) & 1u)) f = pw2[j * kEvalBits + k];
    for (int m = 8; m >= 1; m >>= 1) f = f * shfl_fr(f, l ^ m);
    if (j < NP && k == 0) bpow[j] = f;
  }
  const size_t s = (size_t)blockIdx.x * kT * kEvalChunk2 + threadIdx.x;
  // the Horner sums stay in the 9x29 radix (round 5: no canonical Fr round trip per step):
  // acc < 3r with limbs < 2^30 -> mul29 by y < r gives < (3r r + 2^261 r) / 2^261 < 2r, plus
  // the coefficient (< r) -> < 3r again
  F29 acc[NP];
#pragma unroll
  for (int j = 0; j < NP; j++)
#pragma unroll
    for (int l = 0; l < 9; l++) acc[j].v[l] = 0;
  // from the top coefficient down: indices past a polynomial's length are its top ones, so
  // skipping them (acc still 0) is Horner over zeros
  for (int m = kEvalChunk2 - 1; m >= 0; m--) {
    const size_t i = s + (size_t)m * kT;
#pragma unroll
    for (int j = 0; j < NP; j++)
      if (i < es.len[j]) {
        const F29 t = mul29<Fr29>(acc[j], es.y29[j]), c = split29(es.p[j][i]);
#pragma unroll
        for (int l = 0; l < 9; l++) acc[j].v[l] = t.v[l] + c.v[l];
      }
  }
#pragma unroll
  for (int j = 0; j < NP; j++) {
    const Fr r = block_sum_fr(join_fr29(mul29<Fr29>(acc[j], pw[(size_t)j * kT + threadIdx.x])), sh);
    if (threadIdx.x == 0) bsum[j] = r;
  }
  // (block_sum_fr's barriers made bpow visible) the point j's product in lane j
  if (threadIdx.x < NP) partial[(size_t)threadIdx.x * nblocks + blockIdx.x] = bsum[threadIdx.x] * bpow[threadIdx.x];
}

// block per evaluation: the sum of its workgroups' partial sums
__global__ void __launch_bounds__(kT) k_eval_sum(const Fr* __restrict__ partial, int nblocks, Fr* __restrict__ out) {
  __shared__ Fr sh[kT / 64];
  const int j = blockIdx.x;
  Fr acc = Fr::zero();
  for (int b = (int)threadIdx.x; b < nblocks; b += kT) acc = acc + partial[(size_t)j * nblocks + b];
  const Fr r = block_sum_fr(acc, sh);
  if (threadIdx.x == 0) {
    host_put(out + j, r);  // the mailbox (host memory)
    host_put_done();
  }
}

struct RArgs {
  Fr coefz, coef_ab, ea, eb, ec, coefs3;
};

// Round 4 linearisation polynomial r (n+3 coefficients)
__global__ void k_pol_r(const Fr* __restrict__ pz, const Fr* __restrict__ qm, const Fr* __restrict__ ql,
                        const Fr* __restrict__ qr, const Fr* __restrict__ qo, const Fr* __restrict__ qc,
                        const Fr* __restrict__ s3, size_t n, RArgs r, Fr* __restrict__ out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n + 3) return;
  Fr v = r.coefz * pz[i];
  if (i < n) {
    v = v + r.coef_ab * qm[i] + r.ea * ql[i] + r.eb * qr[i] + r.ec * qo[i] + qc[i];
    v = v - r.coefs3 * s3[i];
  }
  out[i] = v;
}

struct WArgs {
  Fr xim, xi2m, v[7], w0sub;
};

// Round 5 opening polynomial before division (n+6 coefficients)
__global__ void k_pol_wxi(const Fr* __restrict__ t, const Fr* __restrict__ pr, const Fr* __restrict__ pa,
                          const Fr* __restrict__ pb, const Fr* __restrict__ pc, const Fr* __restrict__ s1,
                          const Fr* __restrict__ s2, size_t n, WArgs wa, Fr* __restrict__ out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n + 6) return;
  Fr w = wa.xi2m * t[2 * n + i];
  if (i < n) w = w + wa.xim * t[n + i] + t[i];
  if (i < n + 3) w = w + wa.v[1] * pr[i];
  if (i < n + 2) w = w + wa.v[2] * pa[i] + wa.v[3] * pb[i] + wa.v[4] * pc[i];
  if (i < n) w = w + wa.v[5] * s1[i] + wa.v[6] * s2[i];
  if (i == 0) w = w - wa.w0sub;
  out[i] = w;
}

// "Polinomial does not divide": P0 == -d * q0
__global__ void k_div_check(const Fr* __restrict__ src, Fr p0_adjust, const Fr* __restrict__ q, Fr d,
                            uint32_t* flags, uint32_t bit, uint32_t* __restrict__ mb_flags) {
  if (threadIdx.x || blockIdx.x) return;
  Fr p0 = src[0] - p0_adjust;
  if (!(p0 + d * q[0]).is_zero()) atomicOr(flags, bit);
  host_put(mb_flags, *flags);  // the flags word as of this check, into the mailbox
  host_put_done();
}

__global__ void k_root_table(Fr* __restrict__ out, Fr base, Fr scale, size_t count) {
  // out[i] = scale * base^i, i < count (count <= 4096; one thread per entry)
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  out[i] = scale * pow_u64(base, i);
}

// out[i] = split29(lo[i & 4095] * hi[i >> 12] * scale * 2^5): the per-index factor
// (scale * base^i) as the Montgomery-261 operand of mul_fr29 (NttIo in_f / out_f)
__global__ void k_factor29_table(F29* __restrict__ out, const Fr* __restrict__ lo, const Fr* __restrict__ hi, Fr scale,
                                 size_t count) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  Fr v = lo[i & 4095] * hi[i >> 12] * scale;
#pragma unroll
  for (int k = 0; k < 5; k++) v = v + v;
  out[i] = split29(v);
}

// ----------------------------------------------------------------------------
// host helpers
// ----------------------------------------------------------------------------
static std::string fr_dec(const Fr& m) {
  Fr x = from_mont(m);
  uint32_t v[8];
  std::memcpy(v, x.v, 32);
  std::string s;
  bool nz = true;
  while (nz) {
    uint64_t rem = 0;
    nz = false;
    for (int i = 7; i >= 0; i--) {
      uint64_t cur = (rem << 32) | v[i];
      v[i] = (uint32_t)(cur / 10);
      rem = cur % 10;
      if (v[i]) nz = true;
    }
    s.push_back((char)('0' + rem));
  }
  return std::string(s.rbegin(), s.rend());
}

static Fr fr_small(uint64_t k) {
  Fr x = Fr::zero();
  x.v[0] = (uint32_t)k;
  x.v[1] = (uint32_t)(k >> 32);
  return to_mont(x);
}

Prover::~Prover() {
  for (int i = 0; i < kSlots; i++) {
    if (aux[i]) {
      (void)hipStreamSynchronize(aux[i]);
      (void)hipStreamDestroy(aux[i]);
    }
    if (ready[i]) (void)hipEventDestroy(ready[i]);
  }
  if (side_ready) (void)hipEventDestroy(side_ready);
  if (side_done) (void)hipEventDestroy(side_done);
  if (pows_done) (void)hipEventDestroy(pows_done);
  if (top_host) (void)hipHostFree(top_host);
  for (auto& e : span_ev) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
}

// GPU time spans of the last proof (prof_gpu): a start event before and an end event after
// one transform or one commitment MSM, on the stream it runs on
size_t Prover::span_begin(int kind, hipStream_t s) {
  if (spans_used == span_ev.size()) {
    hipEvent_t a, b;
    NZ_HIP(hipEventCreate(&a));
    NZ_HIP(hipEventCreate(&b));
    span_ev.emplace_back(a, b);
    span_kind.push_back(0);
  }
  span_kind[spans_used] = kind;
  NZ_HIP(hipEventRecord(span_ev[spans_used].first, s));
  return spans_used++;
}
void Prover::span_end(size_t i, hipStream_t s) { NZ_HIP(hipEventRecord(span_ev[i].second, s)); }
void Prover::span_totals(double* msm_ms, double* ntt_ms) {
  *msm_ms = *ntt_ms = 0;
  for (size_t i = 0; i < spans_used; i++) {
    NZ_HIP(hipEventSynchronize(span_ev[i].second));
    float ms = 0;
    NZ_HIP(hipEventElapsedTime(&ms, span_ev[i].first, span_ev[i].second));
    (span_kind[i] ? *ntt_ms : *msm_ms) += ms;
  }
}

MsmShard::~MsmShard() {
  (void)hipSetDevice(device);
  for (auto& s : st)
    if (s) {
      (void)hipStreamSynchronize(s);
      (void)hipStreamDestroy(s);
    }
}

void Prover::set_msm_devices(const std::vector<int>& devices) {
  GuardScope guards;
  if (devices.empty() || devices[0] != eng->device)
    throw Error(NZCB_ERR_ARG, "msm devices must start with the context's device");
  shards.clear();
  own_hi = own_lhi = 0;
  const size_t N = ptau.n;                  // n + 6 bases
  const size_t L = lcommit ? ltau.n : 0;    // n + 2 Lagrange-basis points (A, B, C)
  const size_t k = devices.size();
  if (k == 1) return;
  own_hi = N / k;
  own_lhi = L / k;
  for (size_t i = 1; i < k; i++) {
    auto sh = std::make_unique<MsmShard>();
    sh->device = devices[i];
    sh->lo = N * i / k;
    sh->hi = N * (i + 1) / k;
    sh->llo = L * i / k;
    sh->lhi = L * (i + 1) / k;
    const size_t cnt = sh->hi - sh->lo, lcnt = sh->lhi - sh->llo, mx = std::max(cnt, lcnt);
    NZ_HIP(hipSetDevice(sh->device));
    for (int j = 0; j < MsmShard::kSlots; j++) {
      NZ_HIP(hipStreamCreateWithFlags(&sh->st[j], hipStreamNonBlocking));
      sh->sc[j].reset(new MsmScratch());
      sh->sc[j]->init(mx, true, 1, false);
      sh->scal[j].alloc(mx);
    }
    {  // the shard's PTau range -> its shifted-base table (built on the shard's device)
      DevBuf<G1Affine> part(cnt);
      NZ_HIP(hipMemcpyPeerAsync(part.p, sh->device, ptau.p + sh->lo, eng->device, cnt * sizeof(G1Affine), sh->st[0]));
      sh->table.build(part.p, cnt, fixed_base_window(), sh->st[0]);
      NZ_HIP(hipStreamSynchronize(sh->st[0]));
    }
    if (lcnt) {  // and its range of the Lagrange basis (A, B, C)
      DevBuf<G1Affine> part(lcnt);
      NZ_HIP(hipMemcpyPeerAsync(part.p, sh->device, ltau.p + sh->llo, eng->device, lcnt * sizeof(G1Affine),
                                sh->st[0]));
      sh->ltable.build(part.p, lcnt, lagrange_window(), sh->st[0]);
      sh->ltable.sparse = lagrange_sparse();
      NZ_HIP(hipStreamSynchronize(sh->st[0]));
    }
    shards.push_back(std::move(sh));
  }
  NZ_HIP(hipSetDevice(eng->device));
}

double Prover::ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// ----------------------------------------------------------------------------
// context creation: parse + upload the zkey once
// ----------------------------------------------------------------------------
Prover::Prover(const uint8_t* zkey_bytes, size_t len, int device) {
  GuardScope guards;  // every device buffer of the proving key and lane 0 (common.h)
  Zkey z = parse_zkey(zkey_bytes, len);
  n = z.domainSize;
  n4 = 4 * n;
  power = z.power;
  nVars = z.nVars;
  nPublic = z.nPublic;
  nAdditions = z.nAdditions;
  nConstraints = z.nConstraints;
  if (nAdditions > nVars) throw Error(NZCB_ERR_FORMAT, "nAdditions > nVars");
  nWit = nVars - nAdditions;
  k1 = z.k1;
  k2 = z.k2;
  wn = fr_root_of_unity(power);
  w2 = fr_root_of_unity(2);
  eng.reset(new Engine(device, power + 2, 0));
  init_slots();
  hipStream_t s = st();
  auto up = [&](auto& buf, const Section& sec) {
    using T = typename std::remove_reference<decltype(*buf.p)>::type;
    buf.alloc(sec.len / sizeof(T) ? sec.len / sizeof(T) : 1);
    if (sec.len) NZ_HIP(hipMemcpyAsync(buf.p, sec.p, sec.len, hipMemcpyHostToDevice, s));
  };
  up(ptau, z.ptau);
  // rows of 2^-256 PTau: the commitments' Montgomery-form scalars are digit sources as
  // they are (every ptab MSM is enqueued with mont = true; split ranges and devices keep
  // plain tables)
  ptab.build(ptau.p, ptau.n, fixed_base_window(), s, true);
  lcommit = lagrange_commit_enabled() && ptau.n >= (size_t)n + 2;
  if (lcommit) {  // one elliptic-curve iNTT per context (csrc/lagrange.hip)
    ltau.alloc((size_t)n + 2);
    lagrange_basis(ptau.p, ptau.n, power, ltau.p, s);
    ltab.build(ltau.p, ltau.n, lagrange_window(), s);
    ltab.sparse = lagrange_sparse();
  }
  up(qm, z.qm);
  up(ql, z.ql);
  up(qr, z.qr);
  up(qo, z.qo);
  up(qc, z.qc);
  up(sigma, z.sigma);
  sig_h.alloc((size_t)3 * n);  // sigma_k on H, contiguous (round 2's grand product)
  w_h.alloc(n);                // w^i, i < n (round 2's grand product; built with the root tables below)
  for (int k = 0; k < 3; k++)
    hipLaunchKernelGGL(k_stride4, dim3(grid_for(n, kT, 1u << 30)), dim3(kT), 0, s, sigma.p + (size_t)k * 5 * n + n,
                       (size_t)n, sig_h.p + (size_t)k * n);
  NZ_HIP(hipGetLastError());
  up(lagrange, z.lagrange);
  up(amap, z.amap);
  up(bmap, z.bmap);
  up(cmap, z.cmap);
  // additions: zero out forward references (snarkjs reads not-yet-computed internal
  // signals as 0), then order by dependency level so each level is one parallel launch
  {
    std::vector<uint32_t> level(nAdditions, 0);
    std::vector<AddRec> recs(nAdditions);
    uint32_t maxlev = 0;
    for (uint32_t k = 0; k < nAdditions; k++) {
      const uint8_t* p = z.additions.p + (size_t)k * 72;
      AddRec r;
      std::memcpy(&r.ai, p, 4);
      std::memcpy(&r.bi, p + 4, 4);
      std::memcpy(r.ac.v, p + 8, 32);
      std::memcpy(r.bc.v, p + 40, 32);
      r.dst = nWit + k;
      r.pad = 0;
      uint32_t lv = 0;
      for (uint32_t* ref : {&r.ai, &r.bi}) {
        if (*ref >= nVars) *ref = kZeroRef;
        else if (*ref >= nWit) {
          uint32_t kk = *ref - nWit;
          if (kk >= k) *ref = kZeroRef;
          else lv = std::max(lv, level[kk] + 1);
        }
      }
      level[k] = lv;
      maxlev = std::max(maxlev, lv);
      recs[k] = r;
    }
    std::vector<uint32_t> cnt(maxlev + 2, 0);
    for (uint32_t k = 0; k < nAdditions; k++) cnt[level[k] + 1]++;
    for (uint32_t l = 1; l < cnt.size(); l++) cnt[l] += cnt[l - 1];
    add_level_start.assign(cnt.begin(), cnt.end());
    std::vector<AddRec> sorted(nAdditions);
    std::vector<uint32_t> cur(cnt.begin(), cnt.end());
    for (uint32_t k = 0; k < nAdditions; k++) sorted[cur[level[k]]++] = recs[k];
    adds.alloc(nAdditions ? nAdditions : 1);
    if (nAdditions)
      NZ_HIP(hipMemcpyAsync(adds.p, sorted.data(), nAdditions * sizeof(AddRec), hipMemcpyHostToDevice, s));
    NZ_HIP(hipStreamSynchronize(s));
  }
  // 4n-th roots: w4^i = lo[i & 4095] * hi[i >> 12]
  Fr w4 = fr_root_of_unity(power + 2);
  size_t nlo = 4096, nhi = (n4 + 4095) / 4096;
  const Fr one = Fr::one();
  auto table = [&](DevBuf<Fr>& out, size_t cnt, const Fr& base, const Fr& scale) {
    out.alloc(cnt);
    hipLaunchKernelGGL(k_root_table, dim3(grid_for(cnt, kT)), dim3(kT), 0, s, out.p, base, scale, cnt);
    NZ_HIP(hipGetLastError());
  };
  table(root_lo, nlo, w4, one);
  table(root_hi, nhi, pow_u64(w4, 4096), one);
  hipLaunchKernelGGL(k_root_n, dim3(grid_for(n, kT, 1u << 30)), dim3(kT), 0, s, w_h.p, root_lo.p, root_hi.p,
                     (size_t)n);
  NZ_HIP(hipGetLastError());
  // coset g*<w4>, g = 5 (the Fr multiplicative generator, ffjavascript's nqr): x_i = g*w4^i,
  // g^j and g^-j for coset (un)scaling, and 1/Z_H(x_i) = 1/(g^n w4^(i n) - 1), by i mod 4
  const Fr g = fr_small(5), gi = inverse(g);
  table(x_lo, nlo, w4, g);
  table(g_lo, nlo, g, one);
  table(g_hi, nhi, pow_u64(g, 4096), one);
  table(gi_lo, nlo, gi, one);
  table(gi_hi, nhi, pow_u64(gi, 4096), one);
  quot3 = quot3_enabled() && nPublic <= kQ29MaxPub && power >= 6;
  {  // full per-index coset factors for the NTT prologue (g^j, j < n + 8) and the 4n
     // quotient iNTT's epilogue (g^-j / 4n, j < 4n; not needed by the three-coset quotient)
    const Fr two = one + one;
    g29.alloc((size_t)n + 8);
    hipLaunchKernelGGL(k_factor29_table, dim3(grid_for((size_t)n + 8, kT, 1u << 30)), dim3(kT), 0, s, g29.p, g_lo.p,
                       g_hi.p, one, (size_t)n + 8);
    if (!quot3) {
      gi29.alloc(n4);
      hipLaunchKernelGGL(k_factor29_table, dim3(grid_for(n4, kT, 1u << 30)), dim3(kT), 0, s, gi29.p, gi_lo.p,
                         gi_hi.p, inverse(pow_u64(two, (uint64_t)power + 2)), (size_t)n4);
    }
    NZ_HIP(hipGetLastError());
  }
  {
    Fr gn = pow_u64(g, n), w4n = pow_u64(w4, n), p = gn;
    for (int k = 0; k < 4; k++) {
      zh_inv[k] = inverse(p - one);
      p = p * w4n;
    }
  }
  alloc_workspace();
  if (quot3) {  // the gate check on H reads the selectors on H contiguously (k_gate_h)
    q_h.alloc((size_t)5 * n);
    const DevBuf<Fr>* qs[5] = {&qm, &ql, &qr, &qo, &qc};
    for (int k = 0; k < 5; k++)
      hipLaunchKernelGGL(k_stride4, dim3(grid_for(n, kT, 1u << 30)), dim3(kT), 0, s, qs[k]->p + n, (size_t)n,
                         q_h.p + (size_t)k * n);
    NZ_HIP(hipGetLastError());
  }
  if (quot3) {  // three-coset quotient: per-coset twists c_j^k and untwists c_j^-k / 4n, j < 3
    const size_t nhi3 = (n + 4095) / 4096;
    tw3.alloc((size_t)3 * n);
    itw3.alloc((size_t)3 * n);
    const Fr inv4n = inverse(fr_small(n4));
    DevBuf<Fr> lo, hi;
    for (int j = 0; j < 3; j++) {
      const Fr cj = g * pow_u64(w4, (uint64_t)j), cji = inverse(cj);
      d3[j] = pow_u64(cj, n);
      table(lo, nlo, cj, one);
      table(hi, nhi3, pow_u64(cj, 4096), one);
      hipLaunchKernelGGL(k_factor29_table, dim3(grid_for(n, kT, 1u << 30)), dim3(kT), 0, s, tw3.p + (size_t)j * n,
                         lo.p, hi.p, one, (size_t)n);
      NZ_HIP(hipStreamSynchronize(s));  // lo / hi are reallocated below
      table(lo, nlo, cji, one);
      table(hi, nhi3, pow_u64(cji, 4096), one);
      hipLaunchKernelGGL(k_factor29_table, dim3(grid_for(n, kT, 1u << 30)), dim3(kT), 0, s, itw3.p + (size_t)j * n,
                         lo.p, hi.p, inv4n, (size_t)n);
      NZ_HIP(hipGetLastError());
      NZ_HIP(hipStreamSynchronize(s));
    }
    for (int k = 0; k < 3; k++)
      NZ_HIP(hipMemcpy(sig_top[k], sigma.p + (size_t)k * 5 * n + (n - 4), 4 * sizeof(Fr), hipMemcpyDeviceToHost));
  }
  // coset evaluations of the fixed polynomials from the zkey coefficients (once per context)
  if (quot3) {
    const uint32_t nl = nPublic > 0 ? nPublic : 1;
    const size_t n3 = (size_t)3 * n;
    cq3.alloc(5 * n3);
    cs3.alloc(3 * n3);
    cl3.alloc(nl * n3);
    auto coset3 = [&](const Fr* coefs, Fr* out) {  // Q(c_j w^m) at [j n + m]
      for (int j = 0; j < 3; j++) {
        NttIo io;
        io.in_len = n;
        io.in_f = tw3.p + (size_t)j * n;
        ntt(eng->ntt_tables, coefs, out + (size_t)j * n, power, false, s, nullptr, &io);
      }
    };
    const DevBuf<Fr>* qs[5] = {&qm, &ql, &qr, &qo, &qc};
    for (int k = 0; k < 5; k++) coset3(qs[k]->p, cq3.p + (size_t)k * n3);
    for (int k = 0; k < 3; k++) coset3(sigma.p + (size_t)k * 5 * n, cs3.p + (size_t)k * n3);
    for (uint32_t j = 0; j < nl; j++) coset3(lagrange.p + (size_t)j * 5 * n, cl3.p + (size_t)j * n3);
    NZ_HIP(hipGetLastError());
    auto scale = [&](Fr* p, size_t m, int e) {
      hipLaunchKernelGGL(k_dbl_pow, dim3(grid_for(m, kT, 1u << 30)), dim3(kT), 0, s, p, m, e);
    };
    scale(cq3.p, n3, 10);             // qm
    scale(cq3.p + n3, 3 * n3, 5);     // ql, qr, qo
    scale(cl3.p, (size_t)nl * n3, 5); // L_j
    scale(x_lo.p, nlo, 5);            // g w4^j
    NZ_HIP(hipGetLastError());
  } else {
    const uint32_t nl = nPublic > 0 ? nPublic : 1;
    cq.alloc((size_t)5 * n4);
    cs.alloc((size_t)3 * n4);
    cl.alloc((size_t)nl * n4);
    auto coset_eval = [&](const Fr* coefs, Fr* out) {
      NttIo io;  // coset shift g^j and the zero padding fused into the NTT's first pass
      io.in_len = n;
      io.in_f = g29.p;
      ntt(eng->ntt_tables, coefs, out, power + 2, false, s, nullptr, &io);
    };
    const DevBuf<Fr>* qs[5] = {&qm, &ql, &qr, &qo, &qc};
    for (int k = 0; k < 5; k++) coset_eval(qs[k]->p, cq.p + (size_t)k * n4);
    for (int k = 0; k < 3; k++) coset_eval(sigma.p + (size_t)k * 5 * n, cs.p + (size_t)k * n4);
    for (uint32_t j = 0; j < nl; j++) coset_eval(lagrange.p + (size_t)j * 5 * n, cl.p + (size_t)j * n4);
    NZ_HIP(hipGetLastError());
    if (nPublic <= kQ29MaxPub) {  // exponent pre-scaling of the 29-bit quotient (k_quotient_coset29)
      auto scale = [&](Fr* p, size_t m, int e) {
        hipLaunchKernelGGL(k_dbl_pow, dim3(grid_for(m, kT, 1u << 30)), dim3(kT), 0, s, p, m, e);
      };
      scale(cq.p, n4, 10);                      // qm
      scale(cq.p + n4, 3 * n4, 5);              // ql, qr, qo
      scale(cl.p, (size_t)nl * n4, 5);          // L_j
      scale(x_lo.p, nlo, 5);                    // g w4^j
      NZ_HIP(hipGetLastError());
    }
  }
  NZ_HIP(hipStreamSynchronize(s));
}

void Prover::init_slots() {
  for (int i = 0; i < kSlots; i++) {
    msc[i].reset(new MsmScratch());
    // table schedules only; slot 0 also takes A, B, C's three-set schedule over the Lagrange table
#ifdef NZCB_AB_GENERIC  // A/B (temporary): the generic schedule's arrays allocated too, as before round 6
    msc[i]->init((size_t)n + 6, true, i == 0 ? 3 : 1, true);
#else
    msc[i]->init((size_t)n + 6, true, i == 0 ? 3 : 1, false);
#endif
    NZ_HIP(hipStreamCreateWithFlags(&aux[i], hipStreamNonBlocking));
    NZ_HIP(hipEventCreateWithFlags(&ready[i], hipEventDisableTiming));
  }
  NZ_HIP(hipEventCreateWithFlags(&side_ready, hipEventDisableTiming));
  NZ_HIP(hipEventCreateWithFlags(&side_done, hipEventDisableTiming));
  NZ_HIP(hipEventCreateWithFlags(&pows_done, hipEventDisableTiming));
  mb_apub = kMbEvals + kMbEvalMax;
  mb_pubw = mb_apub + nPublic;
  mb_words = mb_pubw + nPublic;
  // coherent: the kernels' stores reach host memory without a cache writeback
  NZ_HIP(hipHostMalloc((void**)&top_host, mb_words * sizeof(Fr), hipHostMallocCoherent));
  std::memset((void*)top_host, 0, mb_words * sizeof(Fr));
}

// per-proof working set (one per lane)
void Prover::alloc_workspace() {
  wit.alloc(nVars ? nVars : 1);
  wtns_in.alloc(nWit ? nWit : 1);
  A.alloc(n + 2); B.alloc(n + 2); C.alloc(n + 2); Z.alloc(n);
  pol_a.alloc(n + 2); pol_b.alloc(n + 2); pol_c.alloc(n + 2); pol_z.alloc(n + 3);
  // coset evaluations and the quotient: 3n under the three-coset quotient (T also holds
  // round 5's n + 6 Wxi numerator, t the 3n + 6 quotient coefficients), 4n otherwise
  const size_t ne = quot3 ? (size_t)3 * n : n4;
  A4.alloc(ne); B4.alloc(ne); C4.alloc(ne); Z4.alloc(ne);
  T.alloc(ne); Tz.alloc(ne); t.alloc(quot3 ? ne + 6 : n4);
  pol_r.alloc(n + 3); pol_wxi.alloc(n + 6); pol_wxiw.alloc(n + 3);
  blind.alloc(13);  // b1..b11 (index 0 unused), then the 32-bit check flags in slot 12
  // tile totals / heads (n / kTileN + 2) and the small scans' levels over them
  scan_tmp.alloc(3 * ((size_t)n / kTileN + 2) + 64);
  // round 5's divPol1 tables (d = xi, xi w): 2 LinTab, then per d the tile powers Q, Qinv
  lin_qn = (size_t)n / kTileN + 3;
  lin_tab.alloc(2 * sizeof(LinTab) / sizeof(Fr) + 4 * lin_qn);
  lin_host.resize(2 * sizeof(LinTab) / sizeof(Fr));
  size_t nblocks = ((size_t)3 * n + 6 + (size_t)kT * kEvalChunk2 - 1) / ((size_t)kT * kEvalChunk2) + 1;
  eval_part.alloc((size_t)kEvalMax * nblocks + kEvalMax);  // eval_many: kEvalMax rows + results
  // x_j^t, t < kT (F29), then x_j^(4096 2^k), k < kEvalBits (Fr), both from k_eval_pows
  eval_pw.alloc((size_t)kEvalMax * kT + (kEvalMax * kEvalBits * sizeof(Fr) + sizeof(F29) - 1) / sizeof(F29));
  host_part.resize(std::max<size_t>(nblocks, kEvalMax));
  flags.p = (uint32_t*)(blind.p + 12);  // a view: the blinding upload also clears the flags
  flags.n = 1;
  flags.owned = false;
  // Z's interpolation and coset transforms (round 2) run while A, B, C's still use the
  // engine's scratch on aux[2]
  const int zlog = quot3 ? power : power + 2;
  if (zlog > 8) ntt_scr2.alloc((size_t)9 << zlog);
}

// An extra proof lane on the primary's device: shares the HBM-resident proving key
// (zkey sections, shifted PTau table, coset evaluations, root tables) read-only and
// owns its streams, MSM scratch and per-proof working set.
Prover::Prover(const Prover& pk, int lane) {
  GuardScope guards;  // the lane's working set, MSM and NTT scratch (common.h)
  lane_id = lane;
  n = pk.n; n4 = pk.n4; nVars = pk.nVars; nPublic = pk.nPublic; nAdditions = pk.nAdditions;
  nConstraints = pk.nConstraints; nWit = pk.nWit; power = pk.power;
  k1 = pk.k1; k2 = pk.k2; wn = pk.wn; w2 = pk.w2;
  add_level_start = pk.add_level_start;
  transcript_public = pk.transcript_public;
  for (int k = 0; k < 4; k++) zh_inv[k] = pk.zh_inv[k];
  NZ_HIP(hipSetDevice(pk.eng->device));
  eng.reset(new Engine(pk.eng->device, power + 2, 0));
  init_slots();
  ptau.alias(pk.ptau);
  ptab.q.alias(pk.ptab.q);
  ptab.n = pk.ptab.n; ptab.stride = pk.ptab.stride; ptab.c = pk.ptab.c; ptab.nw = pk.ptab.nw;
  ptab.mont_folded = pk.ptab.mont_folded;
  lcommit = pk.lcommit;
  ltau.alias(pk.ltau);
  ltab.q.alias(pk.ltab.q);
  ltab.n = pk.ltab.n; ltab.stride = pk.ltab.stride; ltab.c = pk.ltab.c; ltab.nw = pk.ltab.nw;
  ltab.sparse = pk.ltab.sparse;
  qm.alias(pk.qm); ql.alias(pk.ql); qr.alias(pk.qr); qo.alias(pk.qo); qc.alias(pk.qc);
  sigma.alias(pk.sigma); sig_h.alias(pk.sig_h); q_h.alias(pk.q_h); w_h.alias(pk.w_h); lagrange.alias(pk.lagrange);
  amap.alias(pk.amap); bmap.alias(pk.bmap); cmap.alias(pk.cmap); adds.alias(pk.adds);
  root_lo.alias(pk.root_lo); root_hi.alias(pk.root_hi); x_lo.alias(pk.x_lo);
  g_lo.alias(pk.g_lo); g_hi.alias(pk.g_hi); gi_lo.alias(pk.gi_lo); gi_hi.alias(pk.gi_hi);
  g29.alias(pk.g29); gi29.alias(pk.gi29);
  cq.alias(pk.cq); cs.alias(pk.cs); cl.alias(pk.cl);
  quot3 = pk.quot3;
  cq3.alias(pk.cq3); cs3.alias(pk.cs3); cl3.alias(pk.cl3);
  tw3.alias(pk.tw3); itw3.alias(pk.itw3);
  for (int j = 0; j < 3; j++) d3[j] = pk.d3[j];
  std::memcpy(sig_top, pk.sig_top, sizeof(sig_top));
  alloc_workspace();
}

// ----------------------------------------------------------------------------
// building blocks
// ----------------------------------------------------------------------------
// Round 3 with the quotient on three cosets c_j H (c_j = g w4^j, j < 3) instead of the
// whole 4n coset: deg t <= 3n + 5, so 3n evaluations fix t mod prod_j (X^n - d_j) and the
// six coefficients t[3n..3n+6) come from elsewhere: N = t Z_H gives t[3n + k] = N[4n + k],
// and only the permutation products reach degree 4n, so they are alpha times the top
// coefficients of A B C Z - (A + beta S1)(B + beta S2)(C + beta S3) Z(wX), a convolution of
// the six top coefficients of each factor (host). Per coset one n-point iNTT gives
// t mod (X^n - d_j); k_t_combine solves for the quarters of t. The divisibility check of
// the 4n path (coefficients >= 3n + 6 of the 4n iNTT) becomes the gate check on H.
// Same t, bit for bit: t is unique.
// the gate check on H (t's divisibility, flag bit 1), and the copies t's recombination
// needs: A, B, C's coefficients n-4 .. n+1, Z's n-3 .. n+2 and the flags, into top_host
void Prover::launch_gate_check(hipStream_t s) {
  hipLaunchKernelGGL(k_gate_h, dim3(grid_for(n, kT, 1u << 30)), dim3(kT), 0, s, A.p, B.p, C.p, q_h.p, (size_t)n,
                     nPublic, flags.p);
  NZ_HIP(hipGetLastError());
}

void Prover::copy_tops(hipStream_t s) {
  hipLaunchKernelGGL(k_tops, dim3(1), dim3(32), 0, s, pol_a.p, pol_b.p, pol_c.p, pol_z.p, (size_t)n,
                     (const uint32_t*)flags.p, top_host);
  NZ_HIP(hipGetLastError());
  NZ_HIP(hipStreamSynchronize(s));
  if (top_host[kMbFlags].v[0] & 1u) throw Error(NZCB_ERR_T_DIV, "T Polynomial is not divisible");
}

void Prover::round3_quot3(const Fr& beta, const Fr& gamma, const Fr& alpha, hipStream_t s) {
  const size_t n3 = (size_t)3 * n;
  // Lagrange commitments: round 1 ran the gate check on aux[2] (s waits for side_done), so
  // the one host round trip (tops and flag) comes first, while the GPU is idle anyway, and
  // none sits between the quotient and t's recombination
  const bool side = lcommit;
  if (side) copy_tops(s);
  QArgs29 q29;
  q29.beta = f29_exp(beta, 5);
  q29.k23 = k1 == fr_small(2) && k2 == fr_small(3) ? 1 : 0;
  q29.bk1 = f29_exp(beta * k1, 5);
  q29.bk2 = f29_exp(beta * k2, 5);
  q29.alpha2 = f29_exp(alpha * alpha, 5);
  for (int k = 0; k < 4; k++) q29.zhinv[k] = f29_exp(zh_inv[k], 5);
  q29.gamma = f29_exp(gamma, 0);
  q29.negone = f29_exp(neg(Fr::one()), 0);
  q29.alpha = f29_exp(alpha, 20);
  hipLaunchKernelGGL((k_quotient_coset29<true>), dim3(grid_for(n3, kT, 1u << 30)), dim3(kT), 0, s, A4.p, B4.p, C4.p,
                     Z4.p, cq3.p, cs3.p, cl3.p, nPublic, A.p, (size_t)n, x_lo.p, root_hi.p, q29, T.p);
  if (!side) launch_gate_check(s);
  for (int j = 0; j < 3; j++) {  // v_j = (t mod (X^n - d_j)) / 4
    NttIo io;
    io.out_f = itw3.p + (size_t)j * n;
    io.out_f_has_scale = true;
    {
      const size_t sp = prof_gpu ? span_begin(1, s) : 0;
      ntt(eng->ntt_tables, T.p + (size_t)j * n, Tz.p + (size_t)j * n, power, true, s, nullptr, &io);
      if (prof_gpu) span_end(sp, s);
    }
  }
  NZ_HIP(hipGetLastError());
  if (!side) copy_tops(s);
  Fr top[4][6];  // coefficients n-4 .. n+1 of A, B, C and n-3 .. n+2 of Z
  std::memcpy(top, top_host, sizeof(top));
  // factor coefficients by offset u from the top degree (A, B, C: n + 1; Z: n + 2)
  Fr p1[4][6], p2[4][6];
  const Fr w = wn, wi = inverse(wn);
  const Fr wpow[6] = {w * w, w, Fr::one(), wi, wi * wi, wi * wi * wi};  // w^(2 - u)
  for (int u = 0; u < 6; u++) {
    for (int f3 = 0; f3 < 3; f3++) {
      p1[f3][u] = top[f3][5 - u];
      p2[f3][u] = top[f3][5 - u];
      if (u >= 2) p2[f3][u] = p2[f3][u] + beta * sig_top[f3][5 - u];  // S index n + 1 - u <= n - 1
    }
    p1[3][u] = top[3][5 - u];
    p2[3][u] = top[3][5 - u] * wpow[u];  // Z(wX): coefficient j times w^j
  }
  auto conv = [](const Fr (&x)[6], const Fr (&y)[6], Fr (&out)[6]) {
    for (int s2 = 0; s2 < 6; s2++) {
      Fr acc = Fr::zero();
      for (int u = 0; u <= s2; u++) acc = acc + x[u] * y[s2 - u];
      out[s2] = acc;
    }
  };
  Fr e1[6], e2[6], e3[6], h1[6], h2[6], h3[6];
  conv(p1[0], p1[1], e1);
  conv(e1, p1[2], e2);
  conv(e2, p1[3], e3);
  conv(p2[0], p2[1], h1);
  conv(h1, p2[2], h2);
  conv(h2, p2[3], h3);
  T3Args ta;
  const Fr D = d3[0], D3 = D * D * D, i4 = d3[1] * inverse(D), quarter = inverse(fr_small(4));
  for (int k = 0; k < 6; k++) {
    ta.q3[k] = alpha * (e3[5 - k] - h3[5 - k]);  // t[3n + k] = N[4n + k]
    const Fr c = D3 * ta.q3[k] * quarter;
    ta.c0[k] = c;
    ta.c1[k] = neg(i4 * c);  // (i D)^3 = -i D^3
    ta.c2[k] = neg(c);       // (-D)^3
  }
  ta.i4 = i4;
  ta.two_over_d = fr_small(2) * inverse(D);
  ta.inv_d2 = inverse(D * D);
  hipLaunchKernelGGL(k_t_combine, dim3(grid_for(n, kT, 1u << 30)), dim3(kT), 0, s, Tz.p, (size_t)n, ta, t.p);
  NZ_HIP(hipGetLastError());
}

void Prover::to4t(const Fr* evals, Fr* coefs, Fr* evals4, const int* bidx, int nb, hipStream_t s) {
  if (!s) s = st();
  to4t_coefs(evals, coefs, bidx, nb, s);
  to4t_evals4(coefs, evals4, nb, s);
}

// the blinded coefficients (what the commitment needs) ...
void Prover::to4t_coefs(const Fr* evals, Fr* coefs, const int* bidx, int nb, hipStream_t s, uint32_t* scr) {
  auto t0 = std::chrono::steady_clock::now();
  {
    const size_t sp = prof_gpu ? span_begin(1, s) : 0;
    ntt(eng->ntt_tables, evals, coefs, power, true, s, nullptr, nullptr, scr);
    if (prof_gpu) span_end(sp, s);
  }
  BlindIdx bi;
  bi.count = nb;
  for (int k = 0; k < nb; k++) bi.idx[k] = bidx[k];
  hipLaunchKernelGGL(k_blind, dim3(1), dim3(64), 0, s, coefs, (size_t)n, blind.p, bi);
  NZ_HIP(hipGetLastError());
  ntt_ms += ms_since(t0);  // host enqueue time only (kernels run asynchronously)
}

// ... and their 4n coset evaluations (what round 3's quotient needs)
void Prover::to4t_evals4(const Fr* coefs, Fr* evals4, int nb, hipStream_t s, uint32_t* scr) {
  auto t0 = std::chrono::steady_clock::now();
  // evaluations of the *blinded* polynomial on the coset g*<w4> (round-3 quotient input)
  if (quot3) {  // on c_j H, j < 3: the nb top coefficients folded in (x^n = d_j there)
    for (int j = 0; j < 3; j++) {
      NttIo io;
      io.in_len = n;
      io.in_f = tw3.p + (size_t)j * n;
      io.fold_len = (size_t)nb;
      io.fold_n = n;
      io.fold_f = fr29_operand(d3[j]);
      {
        const size_t sp = prof_gpu ? span_begin(1, s) : 0;
        ntt(eng->ntt_tables, coefs, evals4 + (size_t)j * n, power, false, s, nullptr, &io, scr);
        if (prof_gpu) span_end(sp, s);
      }
    }
    NZ_HIP(hipGetLastError());
    ntt_ms += ms_since(t0);
    return;
  }
  NttIo io;  // coset shift g^j and the zero padding fused into the NTT's first pass
  io.in_len = (size_t)n + nb;
  io.in_f = g29.p;
  {
    const size_t sp = prof_gpu ? span_begin(1, s) : 0;
    ntt(eng->ntt_tables, coefs, evals4, power + 2, false, s, nullptr, &io, scr);
    if (prof_gpu) span_end(sp, s);
  }
  NZ_HIP(hipGetLastError());
  ntt_ms += ms_since(t0);  // host enqueue time only (kernels run asynchronously)
}

// Commitments run on their own streams: the MSM of one polynomial overlaps the NTTs
// of the next and the other MSMs of the same round (their sort / reduction kernels are
// latency-bound and fill the gaps of the compute-bound bucket accumulation).
void Prover::commit_start(int slot, const Fr* coefs, size_t len, const MsmBaseTable* tab, const G1Affine* bases,
                          bool on_main) {
  static const char* const kEnq[kSlots] = {"mark: commit enqueue slot 0", "mark: commit enqueue slot 1",
                                           "mark: commit enqueue slot 2"};
  roctxMarkA(kEnq[slot]);  // host timeline of the commitments (rocprofv3 --marker-trace, tools/timeline.py)
  NZ_HIP(hipEventRecord(ready[slot], st()));
  hipStream_t ms = on_main ? st() : aux[slot];  // the stream this slot's MSM runs on
  if (!on_main) NZ_HIP(hipStreamWaitEvent(ms, ready[slot], 0));
  // Both bases split by point range over the devices / ranks of a split: PTau (the six
  // random-scalar commitments) and, since round 6, the Lagrange basis (A, B, C: mostly small
  // scalars, whose |digit| = 1 bucket a point range divides as well)
  const bool lag = tab != nullptr && tab == &ltab;
  slot_lag[slot] = lag;
  slot_split[slot] = false;
  if (!shards.empty() && (!lag || own_lhi)) {
    for (auto& sh : shards) {
      const size_t lo = lag ? sh->llo : sh->lo, hi = lag ? sh->lhi : sh->hi;
      const size_t cnt = len > lo ? std::min(len, hi) - lo : 0;
      NZ_HIP(hipSetDevice(sh->device));
      if (cnt) {
        NZ_HIP(hipStreamWaitEvent(sh->st[slot], ready[slot], 0));
        NZ_HIP(hipMemcpyPeerAsync(sh->scal[slot].p, sh->device, coefs + lo, eng->device, cnt * sizeof(Fr),
                                  sh->st[slot]));
      }
      msm_enqueue(*sh->sc[slot], nullptr, sh->scal[slot].p, cnt, true, sh->st[slot],
                  lag ? &sh->ltable : &sh->table);  // cnt 0: no-op
    }
    NZ_HIP(hipSetDevice(eng->device));
    len = std::min(len, lag ? own_lhi : own_hi);
    slot_split[slot] = true;
  }
  if (split_send && (!lag || split_own_l)) {  // other ranks take [own, len): hand them the scalars once ready
    NZ_HIP(hipEventSynchronize(ready[slot]));
    if (split_send(split_user, slot | (lag ? NZCB_MSM_LAGRANGE : 0), coefs, len) != 0)
      throw Error(NZCB_ERR_INTERNAL, "msm split: sending the scalars to the other ranks failed");
    len = std::min(len, lag ? split_own_l : split_own);
    slot_split[slot] = true;
  }
  const size_t sp = prof_gpu ? span_begin(0, ms) : 0;
  msm_enqueue(*msc[slot], bases ? bases : ptau.p, coefs, len, true, ms, tab ? tab : &ptab);
  if (prof_gpu) span_end(sp, ms);
  static const bool serial = std::getenv("NZCB_SERIAL") != nullptr;  // profiling: one kernel at a time
  if (serial) NZ_HIP(hipStreamSynchronize(ms));
  static const char* const kDone[kSlots] = {"mark: commit enqueued slot 0", "mark: commit enqueued slot 1",
                                            "mark: commit enqueued slot 2"};
  roctxMarkA(kDone[slot]);
}

namespace {
// 64-byte affine point, x || y as normal-form LE (infinity = zeros): the partials' wire format
void affine_to_le(const G1Affine& a, uint8_t* out) {
  const Fq x = a.is_inf() ? Fq::zero() : from_mont(a.x);
  const Fq y = a.is_inf() ? Fq::zero() : from_mont(a.y);
  std::memcpy(out, x.v, 32);
  std::memcpy(out + 32, y.v, 32);
}

G1xyzz xyzz_from_le(const uint8_t* in) {
  G1Affine a;
  Fq x, y;
  std::memcpy(x.v, in, 32);
  std::memcpy(y.v, in + 32, 32);
  if (x.is_zero() && y.is_zero()) return G1xyzz::inf();
  if (reduce_once(x) != x || reduce_once(y) != y) throw Error(NZCB_ERR_ARG, "msm split: partial not reduced");
  a.x = to_mont(x);
  a.y = to_mont(y);
  return xyzz_from_affine(a);
}
}  // namespace

G1Affine Prover::commit_finish(int slot) {
  auto t0 = std::chrono::steady_clock::now();
  G1xyzz r = msm_finish(*msc[slot], aux[slot]);
  static const char* const kRes[kSlots] = {"mark: commit result slot 0", "mark: commit result slot 1",
                                           "mark: commit result slot 2"};
  roctxMarkA(kRes[slot]);
  const bool split = slot_split[slot];
  for (auto& sh : shards) {  // partial sums of the other devices' point ranges
    if (!split) break;
    NZ_HIP(hipSetDevice(sh->device));
    r = xyzz_add(r, msm_finish(*sh->sc[slot], sh->st[slot]));
  }
  if (!shards.empty()) NZ_HIP(hipSetDevice(eng->device));
  if (split && split_gather) {  // every rank's partial (ours included), added in rank order
    const G1Affine own = xyzz_to_affine(r);
    uint8_t own_le[64];
    affine_to_le(own, own_le);
    std::vector<uint8_t> parts((size_t)split_world * 64);
    if (split_gather(split_user, slot | (slot_lag[slot] ? NZCB_MSM_LAGRANGE : 0), own_le, parts.data()) != 0)
      throw Error(NZCB_ERR_INTERNAL, "msm split: gathering the partial sums failed");
    r = G1xyzz::inf();
    for (int k = 0; k < split_world; k++) r = xyzz_add(r, xyzz_from_le(parts.data() + 64 * (size_t)k));
  }
  msm_ms += ms_since(t0);
  return xyzz_to_affine(r);
}

// A, B and C's commitments in one schedule over the Lagrange table (msm.hip msm_enqueue_sets),
// on the main stream, slot 0's scratch (sized for three sets, init_slots)
void Prover::commit_start_abc(size_t len) {
  roctxMarkA("mark: commit enqueue A, B, C");
  const Fr* sc[3] = {A.p, B.p, C.p};
  const size_t sp = prof_gpu ? span_begin(0, st()) : 0;
  msm_enqueue_sets(*msc[0], sc, 3, len, true, st(), &ltab);
  if (prof_gpu) span_end(sp, st());
  roctxMarkA("mark: commit enqueued A, B, C");
}

void Prover::commit_finish_abc(G1Affine& a, G1Affine& b, G1Affine& c) {
  auto t0 = std::chrono::steady_clock::now();
  G1xyzz r[3];
  msm_finish_sets(*msc[0], st(), r);
  roctxMarkA("mark: commit result A, B, C");
  a = xyzz_to_affine(r[0]);
  b = xyzz_to_affine(r[1]);
  c = xyzz_to_affine(r[2]);
  msm_ms += ms_since(t0);
}

void Prover::set_msm_split(int world, size_t own_points, size_t own_lagrange, nzcb_msm_send_fn send,
                           nzcb_msm_gather_fn gather, void* user) {
  if (world <= 1 || !send || !gather) {
    split_send = nullptr;
    split_gather = nullptr;
    split_world = 1;
    split_own = split_own_l = 0;
    return;
  }
  if (!shards.empty()) throw Error(NZCB_ERR_ARG, "msm split: a context splits over devices or over ranks, not both");
  if (own_points == 0 || own_points > ptau.n) throw Error(NZCB_ERR_ARG, "msm split: bad own point count");
  if (own_lagrange > (lcommit ? ltau.n : 0))
    throw Error(NZCB_ERR_ARG, "msm split: bad own Lagrange point count (A, B, C are committed from coefficients "
                              "when the context has no Lagrange basis)");
  split_send = send;
  split_gather = gather;
  split_user = user;
  split_world = world;
  split_own = own_points;
  split_own_l = own_lagrange;
}

void Prover::eval_many(int np, const Fr* const* polys, const size_t* lens, const Fr* xs, Fr* out,
                       const std::function<void()>& overlap) {
  if (np < 1 || np > kEvalMax) throw Error(NZCB_ERR_INTERNAL, "eval_many: bad count");
  hipStream_t s = st();
  EvalSet es{};
  size_t maxlen = 0;
  for (int j = 0; j < np; j++) {
    es.p[j] = polys[j];
    es.len[j] = lens[j];
    es.x[j] = xs[j];
    es.x29[j] = fr29_operand(xs[j]);
    es.y29[j] = fr29_operand(pow_u64(xs[j], kT));
    es.x4096[j] = pow_u64(xs[j], (uint64_t)kT * kEvalChunk2);
    maxlen = std::max(maxlen, lens[j]);
  }
  es.np = np;
  const size_t nblocks = (maxlen + (size_t)kT * kEvalChunk2 - 1) / ((size_t)kT * kEvalChunk2);
  if (nblocks > ((size_t)1 << kEvalBits)) throw Error(NZCB_ERR_INTERNAL, "eval_many: polynomial too long");
  es.nbits = 1;
  while (((size_t)1 << es.nbits) < nblocks) es.nbits++;
  if ((size_t)np * nblocks + kEvalMax > eval_part.n) throw Error(NZCB_ERR_INTERNAL, "eval partial buffer too small");
  Fr* res = eval_part.p + (size_t)np * nblocks;
  F29* pw = eval_pw.p;
  Fr* pw2 = (Fr*)(eval_pw.p + (size_t)kEvalMax * kT);
  hipLaunchKernelGGL(k_eval_pows, dim3((unsigned)np), dim3(kT), 0, s, es, pw, pw2);
  if (np == 7)
    hipLaunchKernelGGL(k_eval_multi<7>, dim3((unsigned)nblocks), dim3(kT), 0, s, es, (const F29*)pw, (const Fr*)pw2,
                       eval_part.p, (int)nblocks);
  else if (np == 1)
    hipLaunchKernelGGL(k_eval_multi<1>, dim3((unsigned)nblocks), dim3(kT), 0, s, es, (const F29*)pw, (const Fr*)pw2,
                       eval_part.p, (int)nblocks);
  else
    throw Error(NZCB_ERR_INTERNAL, "eval_many: 1 or 7 evaluations");
  NZ_HIP(hipGetLastError());
  (void)res;
  hipLaunchKernelGGL(k_eval_sum, dim3(np), dim3(kT), 0, s, (const Fr*)eval_part.p, (int)nblocks,
                     top_host + kMbEvals);  // the mailbox
  NZ_HIP(hipGetLastError());
  if (overlap) overlap();  // host work beside the evaluation kernels
  NZ_HIP(hipStreamSynchronize(s));
  for (int j = 0; j < np; j++) out[j] = top_host[kMbEvals + j];
}

// divPol1's power tables for d (k_lin_tile's LinTab) into slot k of lin_tab: host products,
// uploaded on stream s (round 4 builds both on aux[2] while its evaluations run)
void Prover::lin_tables(int k, const Fr& d, hipStream_t s) {
  LinTab& t = ((LinTab*)lin_host.data())[k];
  t.dp[0] = Fr::one();
  for (int j = 1; j <= kPer; j++) t.dp[j] = t.dp[j - 1] * d;
  const Fr dk = t.dp[kPer], dki = inverse(dk);  // inverse(0) = 0: Pinv = 0 past t = 0
  t.P[0] = t.Pinv[0] = Fr::one();
  for (int i = 1; i <= kT; i++) {
    t.P[i] = t.P[i - 1] * dk;
    t.Pinv[i] = t.Pinv[i - 1] * dki;
  }
  NZ_HIP(hipMemcpyAsync((LinTab*)lin_tab.p + k, &t, sizeof(LinTab), hipMemcpyHostToDevice, s));
  Fr* q = lin_tile_pows(k);
  const int qn = (int)lin_qn;
  hipLaunchKernelGGL(k_pow_tiles, dim3((qn + 255) / 256), dim3(256), 0, s, t.P[kT], t.Pinv[kT], qn, q, q + qn);
  NZ_HIP(hipGetLastError());
}

Fr* Prover::lin_tile_pows(int k) { return lin_tab.p + 2 * sizeof(LinTab) / sizeof(Fr) + (size_t)k * 2 * lin_qn; }

void Prover::div_pol1(const Fr* src, size_t m, int tab, const Fr& p0_adjust, Fr* dst, uint32_t flag_bit) {
  hipStream_t s = st();
  const size_t ntiles = (m + kTileN - 1) / kTileN;
  const LinTab* lt = (const LinTab*)lin_tab.p + tab;
  const LinTab& ht = ((const LinTab*)lin_host.data())[tab];
  if (ntiles + 1 > lin_qn) throw Error(NZCB_ERR_INTERNAL, "divPol1: more tiles than its power tables");
  Fr* heads = scan_tmp.p;  // ntiles + 1 (the last one 0: the carry into the last tile)
  hipLaunchKernelGGL(k_lin_tile<false>, dim3((unsigned)ntiles), dim3(kT), 0, s, src, m, lt, (const Fr*)nullptr, heads);
  // true heads: H_T = h_T + d^kTileN H_(T+1), by the tile power tables (additions)
  const Fr* q = lin_tile_pows(tab);
  hipLaunchKernelGGL(k_tile_heads, dim3(1), dim3(1024), 0, s, heads, (int)ntiles, q, q + lin_qn);
  NZ_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_lin_tile<true>, dim3((unsigned)ntiles), dim3(kT), 0, s, src, m, lt, (const Fr*)heads, dst);
  hipLaunchKernelGGL(k_div_check, dim3(1), dim3(64), 0, s, src, p0_adjust, dst, ht.dp[1], flags.p, flag_bit,
                     (uint32_t*)(top_host + kMbFlags));
  NZ_HIP(hipGetLastError());
}

// ----------------------------------------------------------------------------
// prove
// ----------------------------------------------------------------------------
// roctx ranges for rocprofv3 --marker-trace (SURVEY.md §5 tracing): "plonk_prove" around
// a proof and one range per phase inside it; exception-safe (the destructor pops).
namespace {
struct RoctxPhases {
  bool open = false;
  explicit RoctxPhases(const char* proof) { roctxRangePush(proof); }
  void next(const char* phase) {
    if (open) roctxRangePop();
    roctxRangePush(phase);
    open = true;
  }
  ~RoctxPhases() {
    if (open) roctxRangePop();
    roctxRangePop();
  }
};
}  // namespace

namespace {
// uniform in [0, r): 254-bit draws from getrandom(2), rejected when >= r
Fr random_fr() {
  for (;;) {
    uint8_t b[32];
    size_t got = 0;
    while (got < sizeof(b)) {
      ssize_t k = getrandom(b + got, sizeof(b) - got, 0);
      if (k < 0) {
        if (errno == EINTR || errno == EAGAIN) continue;  // a signal during the read: draw again
        throw Error(NZCB_ERR_INTERNAL, std::string("getrandom failed: ") + std::strerror(errno) +
                                           " (no entropy for the blinding scalars)");
      }
      got += (size_t)k;
    }
    b[31] &= 0x3f;
    Fr x;
    std::memcpy(x.v, b, 32);
    if (reduce_once(x) == x) return to_mont(x);
  }
}
}  // namespace

void Prover::prove(const uint8_t* witness, size_t n_witness, const uint8_t* blinding, uint8_t* proof_out,
                   uint8_t* pub_out, bool witness_on_device) {
  if (n_witness != nWit) {
    throw Error(NZCB_ERR_WITNESS_LEN, "Invalid witness length. Circuit: " + std::to_string(nVars) +
                                          ", witness: " + std::to_string(n_witness) + ", " +
                                          std::to_string(nAdditions));
  }
  NZ_HIP(hipSetDevice(eng->device));
  hipStream_t s = st();
  msm_ms = ntt_ms = 0;
  spans_used = 0;
  // a previous proof that failed in round 2 may have left the side stream's NTTs running
  // on this lane's buffers (blind, A, B, C)
  if (side_done) NZ_HIP(hipEventSynchronize(side_done));
  // which lane proves (rocprofv3 --marker-trace; tools/lane_speeds.py: lanes differ in speed by
  // the hardware queues their streams landed on, profiles/r6_drain_queues.txt)
  static const char* kLaneMark[17] = {"lane 0", "lane 1", "lane 2", "lane 3", "lane 4", "lane 5", "lane 6", "lane 7",
                                      "lane 8", "lane 9", "lane 10", "lane 11", "lane 12", "lane 13", "lane 14",
                                      "lane 15", "lane 16"};
  roctxMarkA(kLaneMark[lane_id < 16 ? lane_id : 16]);
  RoctxPhases ranges("plonk_prove");
  ranges.next("witness: calculateAdditions + buildABC");
  auto T0 = std::chrono::steady_clock::now();
  auto lg = [&](const std::string& m) { if (log) log(m); };
  // blinding scalars b1..b11 (Montgomery); index 0 unused
  Fr bl[13];
  bl[0] = Fr::zero();
  bl[12] = Fr::zero();  // the check flags (one upload, no fill kernel)
  // NULL blinding: uniform scalars from the OS CSPRNG, as snarkjs's Fr.random() (a proof
  // with zero blinding is not zero-knowledge); callers that want a reproducible proof pass
  // explicit bytes (all zero included)
  for (int i = 1; i <= 11; i++) bl[i] = blinding ? fr_from_le_normal(blinding + 32 * (i - 1)) : random_fr();
  NZ_HIP(hipMemcpyAsync(blind.p, bl, sizeof(bl), hipMemcpyHostToDevice, s));

  lg("Reading Wtns");
  const Fr* wsrc = (const Fr*)witness;
  if (!witness_on_device) {
    NZ_HIP(hipMemcpyAsync(wtns_in.p, witness, (size_t)nWit * 32, hipMemcpyHostToDevice, s));
    wsrc = wtns_in.p;
  } else {
    // a witness in another GPU's HBM (device-set contexts prove one batch on every
    // device): one copy over xGMI into this lane's upload buffer
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, witness) == hipSuccess && at.device != eng->device) {
      NZ_HIP(hipMemcpyPeerAsync(wtns_in.p, eng->device, witness, at.device, (size_t)nWit * 32, s));
      wsrc = wtns_in.p;
    }
  }
  hipLaunchKernelGGL(k_wit_to_mont, dim3(grid_for(nWit, kT, 1u << 30)), dim3(kT), 0, s, wsrc, wit.p,
                     (size_t)nWit);
  for (size_t l = 0; l + 1 < add_level_start.size(); l++) {
    uint32_t a0 = add_level_start[l], a1 = add_level_start[l + 1];
    if (a1 > a0)
      hipLaunchKernelGGL(k_additions, dim3(grid_for(a1 - a0, kT, 1u << 30)), dim3(kT), 0, s, adds.p + a0, a1 - a0,
                         wit.p);
  }
  hipLaunchKernelGGL(k_build_abc, dim3(grid_for(std::max<size_t>(n, nPublic), kT, 1u << 30)), dim3(kT), 0, s,
                     amap.p, bmap.p, cmap.p, nConstraints, n, wit.p, nVars, A.p, B.p, C.p, nPublic,
                     top_host + mb_apub, top_host + mb_pubw);
  NZ_HIP(hipGetLastError());
  NZ_HIP(hipStreamSynchronize(s));
  tm[1] = ms_since(T0);

  // ---------------- round 1 ----------------
  ranges.next("round1: to4T + commit A, B, C");
  auto t1 = std::chrono::steady_clock::now();
  G1Affine pA, pB, pC, pZ, pT1, pT2, pT3, pWxi, pWxiw;
  {
    const int ba[2] = {2, 1}, bb[2] = {4, 3}, bc[2] = {6, 5};
    // one schedule for A, B, C unless the commitments are split over ranks or devices (whose
    // protocol sends each commitment's own scalar ranges)
    const bool abc_sets = lcommit && shards.empty() && !split_send && msc[0]->max_lsets >= 3 && abc_sets_enabled();
    if (lcommit) {
      // evaluations + blinding scalars against the Lagrange basis: the same points, and the
      // MSMs start before the interpolations (they run on the commitment streams)
      hipLaunchKernelGGL(k_abc_tail, dim3(1), dim3(64), 0, s, A.p, B.p, C.p, (size_t)n, blind.p);
      NZ_HIP(hipGetLastError());
      NZ_HIP(hipEventRecord(side_ready, s));  // A, B, C final (k_abc_tail): the side stream's start
      if (abc_sets) {
        // round 6: the three commitments in ONE schedule over the Lagrange table (msm_enqueue_sets:
        // one bucketing, accumulation and carry reduction over 3 x 2^16 buckets, window sums per
        // commitment) on the main stream, instead of three MSMs contending for the chip
        lg("multiexp A");  // snarkjs's logger lines, one per commitment
        lg("multiexp B");
        lg("multiexp C");
        commit_start_abc(n + 2);
      } else {
      lg("multiexp A");
      commit_start(0, A.p, n + 2, &ltab, ltau.p);
      lg("multiexp B");
      commit_start(1, B.p, n + 2, &ltab, ltau.p);
      lg("multiexp C");
      }
      // The interpolations and 4n coset evaluations of A, B, C are only needed by round 3's
      // quotient (and round 4), so they overlap the commitments AND round 2's grand product,
      // which reads the evaluations only (round 2 waits for them before Z's own NTTs, which
      // share the NTT scratch). They run on C's commitment stream, and C's MSM takes the
      // main stream: a stream of their own per lane cost 2.5 % of the 5-lane bench
      // (round 3, profiles/r3_side_stream_ab.txt). msm_finish waits on the MSM's own event,
      // not on its stream.
      hipStream_t ss = aux[2];
      if (!abc_sets) commit_start(2, C.p, n + 2, &ltab, ltau.p, true);
      NZ_HIP(hipStreamWaitEvent(ss, side_ready, 0));
      to4t(A.p, pol_a.p, A4.p, ba, 2, ss);
      to4t(B.p, pol_b.p, B4.p, bb, 2, ss);
      to4t(C.p, pol_c.p, C4.p, bc, 2, ss);
      if (quot3) launch_gate_check(ss);  // t's divisibility from round 1's data (round 3 reads the flag)
      NZ_HIP(hipEventRecord(side_done, ss));
    } else {
      to4t(A.p, pol_a.p, A4.p, ba, 2);
      lg("multiexp A");
      commit_start(0, pol_a.p, n + 2);
      to4t(B.p, pol_b.p, B4.p, bb, 2);
      lg("multiexp B");
      commit_start(1, pol_b.p, n + 2);
      to4t(C.p, pol_c.p, C4.p, bc, 2);
      lg("multiexp C");
      commit_start(2, pol_c.p, n + 2);
    }
    if (lcommit && abc_sets) {
      commit_finish_abc(pA, pB, pC);
    } else {
      pA = commit_finish(0);
      pB = commit_finish(1);
      pC = commit_finish(2);
    }
  }
  tm[2] = ms_since(t1);

  // ---------------- round 2 ----------------
  ranges.next("round2: grand product Z + commit");
  auto t2 = std::chrono::steady_clock::now();
  Fr beta, gamma;
  // A's public-gate values came with k_build_abc (mailbox; the witness phase synchronized)
  const Fr* Apub = top_host + mb_apub;
  {
    std::vector<uint8_t> tr;
    if (transcript_public) {
      for (uint32_t i = 0; i < nPublic; i++) {
        uint8_t be[32];
        fr_to_be(Apub[i], be);
        tr.insert(tr.end(), be, be + 32);
      }
    }
    for (const G1Affine* p : {&pA, &pB, &pC}) {
      uint8_t u[64];
      g1_uncompressed(*p, u);
      tr.insert(tr.end(), u, u + 64);
    }
    beta = hash_to_fr(tr);
    lg("beta: " + fr_dec(beta));
    std::vector<uint8_t> tr2(32);
    fr_to_be(beta, tr2.data());
    gamma = hash_to_fr(tr2);
    lg("gamma: " + fr_dec(gamma));
  }
  {
    PermArgs pa;
    shoup_pair(beta, pa.beta, pa.beta_s);
    shoup_pair(k1 * beta, pa.k1beta, pa.k1beta_s);
    shoup_pair(k2 * beta, pa.k2beta, pa.k2beta_s);
    pa.gamma256 = f29_exp(gamma, 0);
    pa.k23 = k1 == fr_small(2) && k2 == fr_small(3) ? 1 : 0;
    if (fault == NZCB_DEBUG_GENERIC_K) {  // nzcb_debug_inject_fault: the k1, k2 products path, once
      fault = 0;
      pa.k23 = 0;
    }
    const size_t ntiles = (n + kTileN - 1) / kTileN;
    if (ntiles > 1024 * 64) throw Error(NZCB_ERR_INTERNAL, "round 2: domain too large for the tile factors");
    Fr* ntot = scan_tmp.p;  // per tile: numerator / denominator totals, then the factors F_T
    Fr* dtot = ntot + ntiles;
    Fr* fac = dtot + ntiles;
    Fr* totals = fac + ntiles;
    hipLaunchKernelGGL(k_perm_tile, dim3((unsigned)ntiles), dim3(kT), 0, s, A.p, B.p, C.p, sig_h.p, (size_t)n,
                       w_h.p, pa, Z.p, ntot, dtot);
    hipLaunchKernelGGL(k_perm_factors, dim3(1), dim3(1024), 0, s, (const Fr*)ntot, (const Fr*)dtot, (int)ntiles,
                       fac, top_host + kMbTotals);
    NZ_HIP(hipGetLastError());
    // Z[n] = prod num / prod den must be 1; 1 / prod den scales the tiles
    NZ_HIP(hipStreamSynchronize(s));
    const Fr tt[2] = {top_host[kMbTotals], top_host[kMbTotals + 1]};
    if (tt[0] != tt[1]) throw Error(NZCB_ERR_COPY, "Copy constraints does not match");
    hipLaunchKernelGGL(k_apply_tiles, dim3((unsigned)ntiles), dim3(kT), 0, s, Z.p, (size_t)n,
                       (const Fr*)fac, inverse(tt[1]));
    NZ_HIP(hipGetLastError());
    const int bz[3] = {9, 8, 7};
    // Z's transforms use their own scratch (ntt_scr2), so they need not wait for A, B, C's
    // on aux[2] (round 3 does). Z's commitment needs only its coefficients: its MSM starts
    // before the coset NTTs, which run beside it on the main stream (single-proof round 2: -1 ms)
    to4t_coefs(Z.p, pol_z.p, bz, 3, s, ntt_scr2.p);
    lg("multiexp Z");
    commit_start(0, pol_z.p, n + 3);
    to4t_evals4(pol_z.p, Z4.p, 3, s, ntt_scr2.p);
    pZ = commit_finish(0);
  }
  tm[3] = ms_since(t2);

  // ---------------- round 3 ----------------
  ranges.next("round3: quotient t + commit T1, T2, T3");
  auto t3 = std::chrono::steady_clock::now();
  Fr alpha;
  {
    std::vector<uint8_t> tr(64);
    g1_uncompressed(pZ, tr.data());
    alpha = hash_to_fr(tr);
    lg("alpha: " + fr_dec(alpha));
  }
  {
    QArgs q;
    q.beta = beta;
    q.gamma = gamma;
    q.alpha = alpha;
    q.alpha2 = alpha * alpha;
    q.bk1 = beta * k1;
    q.bk2 = beta * k2;
    for (int k = 0; k < 4; k++) q.zhinv[k] = zh_inv[k];
    auto tq = std::chrono::steady_clock::now();
    NZ_HIP(hipStreamWaitEvent(s, side_done, 0));  // A, B, C's coset evaluations (aux[2], round 1)
    if (quot3) {
      round3_quot3(beta, gamma, alpha, s);
    } else if (nPublic <= kQ29MaxPub) {
      QArgs29 q29;
      q29.beta = f29_exp(beta, 5);
      q29.k23 = k1 == fr_small(2) && k2 == fr_small(3) ? 1 : 0;
      q29.bk1 = f29_exp(q.bk1, 5);
      q29.bk2 = f29_exp(q.bk2, 5);
      q29.alpha2 = f29_exp(q.alpha2, 5);
      for (int k = 0; k < 4; k++) q29.zhinv[k] = f29_exp(zh_inv[k], 5);
      q29.gamma = f29_exp(gamma, 0);
      q29.negone = f29_exp(neg(Fr::one()), 0);
      q29.alpha = f29_exp(alpha, 20);
      hipLaunchKernelGGL((k_quotient_coset29<false>), dim3(grid_for(n4, kT, 1u << 30)), dim3(kT), 0, s, A4.p, B4.p,
                         C4.p, Z4.p, cq.p, cs.p, cl.p, nPublic, A.p, (size_t)n, x_lo.p, root_hi.p, q29, T.p);
    } else {
      hipLaunchKernelGGL(k_quotient_coset, dim3(grid_for(n4, kT, 1u << 30)), dim3(kT), 0, s, A4.p, B4.p, C4.p,
                         Z4.p, cq.p, cs.p, cl.p, nPublic, A.p, (size_t)n, x_lo.p, root_hi.p, q, T.p);
    }
    NZ_HIP(hipGetLastError());
    if (!quot3) {
      NttIo io;  // 1/4n, the coset unscale g^-j and the degree check fused into the iNTT's last pass
      io.out_f = gi29.p;
      io.out_f_has_scale = true;
      io.out_limit = (size_t)3 * n + 6;
      io.out_flags = flags.p;
      {
        const size_t sp = prof_gpu ? span_begin(1, s) : 0;
        ntt(eng->ntt_tables, T.p, t.p, power + 2, true, s, nullptr, &io);
        if (prof_gpu) span_end(sp, s);
      }
      NZ_HIP(hipGetLastError());
      uint32_t f = 0;
      NZ_HIP(hipMemcpyAsync(&f, flags.p, 4, hipMemcpyDeviceToHost, s));
      NZ_HIP(hipStreamSynchronize(s));
      if (f & 1u) throw Error(NZCB_ERR_T_DIV, "T Polynomial is not divisible");
    }
    ntt_ms += ms_since(tq);
    if (fault == NZCB_FAULT_QUOTIENT) {  // nzcb_debug_inject_fault: t[1] += 1, once
      fault = 0;
      hipLaunchKernelGGL(k_fault_bump, dim3(1), dim3(64), 0, s, t.p + 1);
      NZ_HIP(hipGetLastError());
    }
    lg("multiexp T1");
    commit_start(0, t.p, n);
    lg("multiexp T2");
    commit_start(1, t.p + n, n);
    lg("multiexp T3");
    commit_start(2, t.p + 2 * (size_t)n, n + 6);
    pT1 = commit_finish(0);
    pT2 = commit_finish(1);
    pT3 = commit_finish(2);
  }
  tm[4] = ms_since(t3);

  // ---------------- round 4 ----------------
  ranges.next("round4: evaluations");
  auto t4 = std::chrono::steady_clock::now();
  Fr xi, ea, eb, ec, es1, es2, et, ezw, er, xim;
  {
    std::vector<uint8_t> tr(192);
    g1_uncompressed(pT1, tr.data());
    g1_uncompressed(pT2, tr.data() + 64);
    g1_uncompressed(pT3, tr.data() + 128);
    xi = hash_to_fr(tr);
    lg("xi: " + fr_dec(xi));
    {
      const Fr* polys[7] = {pol_a.p, pol_b.p, pol_c.p, sigma.p, sigma.p + 5 * (size_t)n, t.p, pol_z.p};
      const size_t lens[7] = {n + 2, n + 2, n + 2, n, n, 3 * (size_t)n + 6, n + 3};
      const Fr xs[7] = {xi, xi, xi, xi, xi, xi, xi * wn};
      Fr ev[7];
      // round 5's divPol1 tables (d = xi, xi w) on the host while the evaluations run
      eval_many(7, polys, lens, xs, ev, [&] {
        lin_tables(0, xi, aux[2]);
        lin_tables(1, xi * wn, aux[2]);
        NZ_HIP(hipEventRecord(pows_done, aux[2]));
      });
      NZ_HIP(hipStreamWaitEvent(s, pows_done, 0));  // round 5's divPol1 reads them
      ea = ev[0];
      eb = ev[1];
      ec = ev[2];
      es1 = ev[3];
      es2 = ev[4];
      et = ev[5];
      ezw = ev[6];
    }
    Fr coef_ab = ea * eb;
    Fr betaxi = beta * xi;
    Fr e2 = (ea + betaxi + gamma) * (eb + betaxi * k1 + gamma);
    e2 = e2 * (ec + betaxi * k2 + gamma) * alpha;
    Fr e3 = (ea + beta * es1 + gamma) * (eb + beta * es2 + gamma);
    e3 = e3 * beta * ezw * alpha;
    xim = xi;
    for (int i = 0; i < power; i++) xim = sqr(xim);
    Fr eval_l1 = (xim - Fr::one()) * inverse((xi - Fr::one()) * fr_small(n));
    Fr e4 = eval_l1 * (alpha * alpha);
    RArgs ra{e2 + e4, coef_ab, ea, eb, ec, e3};
    hipLaunchKernelGGL(k_pol_r, dim3(grid_for(n + 3, kT, 1u << 30)), dim3(kT), 0, s, pol_z.p, qm.p, ql.p, qr.p,
                       qo.p, qc.p, sigma.p + 10 * (size_t)n, (size_t)n, ra, pol_r.p);
    NZ_HIP(hipGetLastError());
    {
      const Fr* polys[1] = {pol_r.p};
      const size_t lens[1] = {n + 3};
      eval_many(1, polys, lens, &xi, &er);
    }
    // The quotient checked at xi before it is committed to: the three-coset t
    // is never inverse-transformed over 4n, so nothing else would catch an error in its
    // coset evaluations, t's recombination or the round-3 stream ordering. From the round-4
    // evaluations (what plonk_verify recomputes): t(xi) Z_H(xi) = r(xi) + PI(xi)
    //   - alpha (a + b s1 + g)(b + b s2 + g)(c + g) z(w xi) - alpha^2 L1(xi)
    // with PI(xi) = -sum_j pub_j L_j(xi), L_j(xi) = w^j (xi^n - 1) / (n (xi - w^j)).
    {
      const Fr zh = xim - Fr::one(), nf = fr_small(n);
      Fr pi = Fr::zero(), wj = Fr::one();
      for (uint32_t j = 0; j < nPublic; j++) {
        pi = pi - Apub[j] * wj * zh * inverse(nf * (xi - wj));
        wj = wj * wn;
      }
      const Fr perm = alpha * (ea + beta * es1 + gamma) * (eb + beta * es2 + gamma) * (ec + gamma) * ezw;
      if (et * zh != er + pi - perm - e4)
        throw Error(NZCB_ERR_INTERNAL, "quotient check failed: t(xi) Z_H(xi) differs from the numerator at xi");
    }
  }
  tm[5] = ms_since(t4);

  // ---------------- round 5 ----------------
  ranges.next("round5: Wxi, Wxiw + commit");
  auto t5 = std::chrono::steady_clock::now();
  {
    std::vector<uint8_t> tr(7 * 32);
    const Fr* ev[7] = {&ea, &eb, &ec, &es1, &es2, &ezw, &er};
    for (int i = 0; i < 7; i++) fr_to_be(*ev[i], tr.data() + 32 * i);
    WArgs wa;
    wa.v[0] = Fr::zero();
    wa.v[1] = hash_to_fr(tr);
    lg("v: " + fr_dec(wa.v[1]));
    for (int i = 2; i <= 6; i++) wa.v[i] = wa.v[i - 1] * wa.v[1];
    wa.xim = xim;
    wa.xi2m = xim * xim;
    wa.w0sub = et + wa.v[1] * er + wa.v[2] * ea + wa.v[3] * eb + wa.v[4] * ec + wa.v[5] * es1 + wa.v[6] * es2;
    hipLaunchKernelGGL(k_pol_wxi, dim3(grid_for(n + 6, kT, 1u << 30)), dim3(kT), 0, s, t.p, pol_r.p, pol_a.p,
                       pol_b.p, pol_c.p, sigma.p, sigma.p + 5 * (size_t)n, (size_t)n, wa, T.p);
    NZ_HIP(hipGetLastError());
    div_pol1(T.p, n + 6, 0, Fr::zero(), pol_wxi.p, 4u);
    lg("multiexp Wxi");
    commit_start(0, pol_wxi.p, n + 6);
    div_pol1(pol_z.p, n + 3, 1, ezw, pol_wxiw.p, 4u);
    lg("multiexp Wxiw");
    commit_start(1, pol_wxiw.p, n + 3);
    NZ_HIP(hipStreamSynchronize(s));  // the two division checks' flags are in the mailbox
    const uint32_t f = top_host[kMbFlags].v[0];
    pWxi = commit_finish(0);
    pWxiw = commit_finish(1);
    if (f & 4u) throw Error(NZCB_ERR_DIVPOL, "Polinomial does not divide");
  }
  tm[6] = ms_since(t5);
  tm[0] = ms_since(T0);
  tm[7] = msm_ms;
  tm[8] = ntt_ms;
  tm[9] = tm[10] = -1;  // not measured
  if (prof_gpu) span_totals(&tm[9], &tm[10]);

  // ---------------- output ----------------
  const G1Affine* pts[9] = {&pA, &pB, &pC, &pZ, &pT1, &pT2, &pT3, &pWxi, &pWxiw};
  for (int i = 0; i < 9; i++) {
    uint8_t* o = proof_out + 64 * i;
    if (pts[i]->is_inf()) {
      std::memset(o, 0, 64);
    } else {
      Fq x = from_mont(pts[i]->x), y = from_mont(pts[i]->y);
      std::memcpy(o, x.v, 32);
      std::memcpy(o + 32, y.v, 32);
    }
  }
  const Fr* ev[7] = {&ea, &eb, &ec, &es1, &es2, &ezw, &er};
  for (int i = 0; i < 7; i++) fr_to_le_normal(*ev[i], proof_out + 9 * 64 + 32 * i);
  for (uint32_t i = 0; i < nPublic; i++) {
    // publicSignals = witness[1..nPublic] (normal form, reduced): k_build_abc wrote their
    // Montgomery forms into the mailbox
    fr_to_le_normal(top_host[mb_pubw + i], pub_out + 32 * (size_t)i);
  }
}

}  // namespace nzcb
