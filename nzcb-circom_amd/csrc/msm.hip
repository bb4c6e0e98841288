// BN254 G1 multi-scalar multiplication for gfx950 (Pippenger, signed windows).
//
// Replaces ffjavascript G1.multiExpAffine + wasmcurves g1m_multiexpAffine_chunk
// (/root/reference/yarn.lock:3905-3913, 8173-8179), which
// split the points into chunks and the scalar bits into pTSizes[log2 n] windows
// (16 bits at 2^21) on CPU workers. The result is a unique group element, so
// any correct schedule is bit-exact after conversion to affine.
//
// Two schedules share the kernels:
//  * generic (variable bases): c-bit windows, one bucket set per window
//    (key = window * 2^(c-1) + |digit| - 1), host Horner over the windows;
//  * fixed-base (the prover's PTau): a table of shifted bases 2^(c*w) * B_i
//    (MsmBaseTable) turns the windows into ONE set of 2^(c-1) buckets (key =
//    |digit| - 1, value = row w of the table) and a single bucket reduction. c = 17
//    by default (15 rows, 2^16 buckets): measured against c = 16..20 at 2^21, it
//    balances the bucket additions (15 per scalar) with the reduction tail. Its accumulation runs in
//    the carry-free 9 x 29-bit radix of csrc/f29.h (table stored Montgomery-261).
//
// Pipeline (one stream, no host sync until the bucket-set sums):
//  1. keys:       thread per scalar -> signed c-bit digits; (scalar, window) pair i
//                 gets the fixed slot w*n+i; zero digits get a sentinel key that
//                 sorts last (or, with 16-bit fixed-base keys, bucket 0 and the
//                 table's infinity point) -- no atomics
//  2. sort:       rocPRIM onesweep radix sort of (key, base index|sign), 2 passes of
//                 <= 10 key bits (16-bit keys for the fixed-base c <= 17)
//  3. offsets:    bucket start positions by binary search in the sorted keys
//  4. accumulate: thread per fixed 48-entry chunk of the sorted stream (doubled past
//                 2^26 entries, chunk_for; load balance
//                 independent of the digit distribution): XYZZ mixed adds of the
//                 gathered affine bases; bucket runs inside one chunk are written
//                 directly, runs crossing a chunk edge go to per-chunk carries
//  5. finalize:   thread per bucket spanning chunks: owner carry + continuations
//  6. reduce:     thread per (set, 8-bucket segment): running sum / weighted sum
//  7. sums:       slot 0 sums the segments' weighted sums, slot b+1 sums the running
//                 sums of segments whose index has bit b set (the segment-offset
//                 weights, in binary); two levels of block tree sums
//  8. host:       per set W = T + 8 * sum_b 2^b R_b, then Horner over the sets
// Generic bases are read straight from the zkey PTau layout (64 B LEM affine).
#include "msm.h"

#include "f29.h"

#include <atomic>
#include <type_traits>
#include <cstdlib>
#include <rocprim/rocprim.hpp>

namespace nzcb {

static constexpr int kMsmThreads = 256;

// Onesweep with a chosen digit width: the generic path's 20-bit keys take 2 passes of
// 10 bits instead of 3 with the library's 8-bit default for gfx950.
#ifndef NZ_SORT_BLOCK
#define NZ_SORT_BLOCK 1024
#endif
#ifndef NZ_SORT_ITEMS
#define NZ_SORT_ITEMS 16
#endif
template <unsigned Bits>
using SortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<NZ_SORT_BLOCK, NZ_SORT_ITEMS>,
                                        rocprim::kernel_config<NZ_SORT_BLOCK, NZ_SORT_ITEMS>, Bits,
                                        rocprim::block_radix_rank_algorithm::match>>;

// digit bits per onesweep pass: 8 for 16-bit keys, 10 for the <= 20-bit 32-bit keys
// (measured at 2^21: 0.51 vs 0.62 ms and 0.55 vs 0.69 ms); NZCB_SORT_BITS overrides
static int sort_bits(bool k16) {
  static const int env = [] {
    const char* e = std::getenv("NZCB_SORT_BITS");
    const int b = e ? std::atoi(e) : 0;
    return (b == 8 || b == 10 || b == 11) ? b : 0;
  }();
  return env ? env : k16 ? 8 : 10;
}

template <class K>
static void radix_sort(void* tmp, size_t& tmp_bytes, const K* kin, K* kout, const uint32_t* vin,
                       uint32_t* vout, size_t m, int end_bit, hipStream_t st) {
  switch (sort_bits(sizeof(K) == 2)) {
    case 8:
      NZ_HIP(rocprim::radix_sort_pairs<SortConfig<8>>(tmp, tmp_bytes, kin, kout, vin, vout, m, 0, end_bit, st));
      break;
    case 11:
      NZ_HIP(rocprim::radix_sort_pairs<SortConfig<11>>(tmp, tmp_bytes, kin, kout, vin, vout, m, 0, end_bit, st));
      break;
    default:
      NZ_HIP(rocprim::radix_sort_pairs<SortConfig<10>>(tmp, tmp_bytes, kin, kout, vin, vout, m, 0, end_bit, st));
  }
}
// entries per accumulation thread, up to 2^26 entries: 48 cuts the carries the finalize
// adds by a third against 32 (same box: bench 32.5 -> 32.9 proofs/s; isolated
// accumulate + finalize 2.8 ms for 32, 40 and 48, 2.9 ms for 64, whose 1.9 rounds of
// waves leave a tail)
static constexpr uint32_t kChunk = 48;
static constexpr uint32_t kMinChunk = 32;  // NZCB_ACC_CHUNK lower bound (carry buffers are sized by it)

// Entries per accumulation thread: kChunk up to 2^26 entries, then doubled so the grid
// stays ~2^19-2^20 threads and a bucket spans ~10 chunks at every size (at 2^24 points a
// fixed 32-entry chunk left ~120 carries per bucket and the finalize took 360 ms).
static uint32_t chunk_for(size_t entries) {
  static const uint32_t base = [] {  // NZCB_ACC_CHUNK: A/B measurements of the chunk size
    const char* e = std::getenv("NZCB_ACC_CHUNK");
    const int v = e ? std::atoi(e) : 0;
    return v >= (int)kMinChunk && v <= 256 ? (uint32_t)v : kChunk;
  }();
  uint32_t c = base;
  while (entries / c > (size_t(1) << 20)) c *= 2;
  return c;
}
static constexpr int kPairThreads = 256;  // pairing rounds: workgroup (one inversion each)
static constexpr int kPairPer = 64;       // pairing rounds: pair slots per thread
static constexpr int kMaxPairRounds = 6;
static constexpr int kSegLen = 8;
static constexpr int kSumThreads = 256;  // level-1 sums: block size
static constexpr int kSumPer = 4;        // level-1 sums: sequential adds per thread
static constexpr int kPartThreads = 64;  // level-2 sums: block size
static constexpr uint32_t kSeqSpan = 64;  // finalize: longest carry run summed by one thread
// the same for the fixed-base (radix 2^29) carries: at 2^21 random scalars a bucket spans
// ~11 chunks; the Lagrange-basis commitments' skewed digits leave a few hundred buckets
// with 17..1000s of carries, and a thread walking 64 of them sequentially was the
// finalize's long pole (0.8 ms per launch, profiles/r3_single_lane_phases.txt)
static constexpr uint32_t kSeqSpan29 = 16;
static constexpr int kLargeBlocks = 32;  // finalize: workgroups for the longer runs
static constexpr int kFbWindow = 17;     // fixed-base window of the PTau tables (NZCB_FB_WINDOW)
// fixed base: workgroups over the pieces of the longer runs, and over their buckets (grid-
// stride; random scalars list none, and under 5 proof lanes every launched workgroup waits
// for a CU slot first, so the grids are kept small)
static constexpr int kLargePieceBlocks = 128;
static constexpr int kLargeFinalBlocks = 128;
static constexpr int kLargeFinalThreads = 64;

// LDS-staged bucket indices in the accumulation (msm_accumulate29_kernel kLdsIdx);
// NZCB_ACC_LDS=0 reads them from HBM as before (A/B runs)
static bool lds_indices() {
  static const bool on = [] {
    const char* e = std::getenv("NZCB_ACC_LDS");
    return !(e && e[0] == '0');
  }();
  return on;
}

// the 4-wave accumulation with LDS-DMA point prefetch (msm_accumulate29_dma_kernel);
// NZCB_ACC_DMA=1 for A/B runs
static bool acc_dma() {
  static const bool on = [] {
    const char* e = std::getenv("NZCB_ACC_DMA");
    return e && e[0] == '1';
  }();
  return on;
}

// the run's second addition without the products by ZZ1 = ZZZ1 = 1 (kAff); NZCB_ACC_AFF=1
static bool acc_aff() {
  static const bool on = [] {
    const char* e = std::getenv("NZCB_ACC_AFF");
    return e && e[0] == '1';
  }();
  return on;
}

// interleaved product pairs in the accumulation (kPair); NZCB_ACC_PAIR=0 for A/B runs
// (same box: isolated accumulation 2.295 -> 2.254 ms, bench +1.3 %)
static bool paired_products() {
  static const bool on = [] {
    const char* e = std::getenv("NZCB_ACC_PAIR");
    return !(e && e[0] == '0');
  }();
  return on;
}
// fixed base, the window sum sum_k (k + 1) B_k (NZCB_FB_SUMS, for A/B runs):
//   2 (default) segments of kSeg29 buckets + bit-slot sums, radix 2^29 (msm_seg29_kernel)
//   1           bit slots over the buckets themselves (msm_bitsums29_kernel)
//   0           the generic schedule's 8x32 segment reduce + slot sums
// Same box (profiles/r3_fb_sums_ab.txt): 1 cut the isolated MSM 3.48 -> 3.08 ms but moved
// 4x the additions of 0 (every bucket in ~8 slots) and the 5-lane bench lost 2 %.
static uint32_t seq_span29() {  // NZCB_SEQ_SPAN29: longest carry run a finalize thread sums (A/B)
  static const uint32_t v = [] {
    const char* e = std::getenv("NZCB_SEQ_SPAN29");
    const int x = e ? std::atoi(e) : (int)kSeqSpan29;
    return (uint32_t)(x >= 1 ? x : kSeqSpan29);
  }();
  return v;
}

static bool lo_split() {  // NZCB_LO_SPLIT=0: one workgroup per high-byte region (A/B runs)
  static const bool on = [] {
    const char* e = std::getenv("NZCB_LO_SPLIT");
    return !(e && e[0] == '0');
  }();
  return on;
}

static bool lo_agg() {  // NZCB_LO_AGG=1: wave-aggregated LDS atomics in msm_lo_* (A/B runs)
  static const bool on = [] {
    const char* e = std::getenv("NZCB_LO_AGG");
    return e && e[0] == '1';
  }();
  return on;
}

static int fin_lanes() {  // NZCB_FIN_LANES=4: msm_finalize29_kernel (latency), else sequential
  static const int v = [] {
    const char* e = std::getenv("NZCB_FIN_LANES");
    return e ? std::atoi(e) : 1;
  }();
  return v;
}

static int fb_sums() {
  static const int v = [] {
    const char* e = std::getenv("NZCB_FB_SUMS");
    const int x = e ? std::atoi(e) : 2;
    return x >= 0 && x <= 2 ? x : 2;
  }();
  return v;
}

int fixed_base_window() {
  static const int c = [] {
    const char* e = std::getenv("NZCB_FB_WINDOW");
    const int v = e ? std::atoi(e) : kFbWindow;
    return (v >= 16 && v <= 20) ? v : kFbWindow;
  }();
  return c;
}

int lagrange_window() {
  static const int c = [] {
    const char* e = std::getenv("NZCB_LB_WINDOW");
    const int v = e ? std::atoi(e) : 17;
    return (v >= 16 && v <= 20) ? v : 17;
  }();
  return c;
}

// Pairing rounds (msm_pair29_kernel) before the fixed-base accumulation: -1 = automatic
// (NZCB_PAIR_ROUNDS rounds while the average bucket run is >= 8 entries; default 0, see
// at 2^21 one round costs 2.9 ms against 2.35 ms for the whole XYZZ
// accumulation), >= 0 = exactly that many (nzcb_msm_set_pair_rounds, tests).
static std::atomic<int> g_pair_rounds{-1};
void msm_set_pair_rounds(int r) { g_pair_rounds.store(r < 0 ? -1 : (r > kMaxPairRounds ? kMaxPairRounds : r)); }

static int pair_rounds_for(size_t entries, uint32_t nkeys) {
  const int forced = g_pair_rounds.load();
  if (forced >= 0) return forced;
  static const int dflt = [] {
    const char* e = std::getenv("NZCB_PAIR_ROUNDS");
    const int v = e ? std::atoi(e) : 0;
    return v < 0 ? 0 : (v > kMaxPairRounds ? kMaxPairRounds : v);
  }();
  int r = 0;
  while (r < dflt && (entries >> r) >= (size_t)8 * nkeys) r++;
  return r;
}

// upper bound of the entries left after a pairing round: sum_k ceil(L_k / 2)
static size_t pair_bound(size_t entries, uint32_t nkeys) { return std::min(entries, (entries + nkeys) / 2); }
static size_t pair_grid(size_t slots) {
  const size_t per = (size_t)kPairThreads * kPairPer;
  return std::max<size_t>(1, (slots + per - 1) / per);
}

int msm_window_bits(size_t n) {
  if (n >= (size_t(1) << 18)) return 16;
  int lg = ilog2(n ? n : 1);
  int c = lg - 3;
  if (c < 4) c = 4;
  if (c > 16) c = 16;
  return c;
}

static inline int num_windows(int c) { return (255 + c - 1) / c; }

template <int C, class F>
__device__ __forceinline__ void for_each_digit(const Fr& s, F&& f) {
  constexpr int NW = (255 + C - 1) / C;
  constexpr uint32_t MASK = (1u << C) - 1u;
  constexpr uint32_t HALF = 1u << (C - 1);
  uint32_t carry = 0;
#pragma unroll
  for (int w = 0; w < NW; w++) {
    const int bit = w * C;
    const int limb = bit >> 5;
    const int sh = bit & 31;
    uint64_t x = s.v[limb];
    if (limb + 1 < 8) x |= (uint64_t)s.v[limb + 1] << 32;
    uint32_t d = ((uint32_t)(x >> sh) & MASK) + carry;
    if (d > HALF) {
      uint32_t mag = (MASK + 1u) - d;
      if (mag) f(w, mag - 1u, 1u);
      carry = 1;
    } else {
      if (d) f(w, d - 1u, 0u);
      carry = 0;
    }
  }
}

// FIXED: key = bucket, value = table row w (stride) + i; else key = w * NB + bucket, value = i.
// Zero digits: with 16-bit keys (fixed base, c <= 17) key 0 and the table's infinity
// point as value (the accumulation skips it), so the keys stay 16 bits; otherwise a
// sentinel key that sorts after every bucket.
template <int C, bool FIXED, class K>
__global__ void __launch_bounds__(kMsmThreads)
msm_keys_kernel(const Fr* __restrict__ scalars, size_t n, int mont, size_t stride, uint32_t skip_val,
                K* __restrict__ keys, uint32_t* __restrict__ vals) {
  constexpr int NW = (255 + C - 1) / C;
  constexpr uint32_t NB = 1u << (C - 1);
  constexpr bool K16 = sizeof(K) == 2;
  static_assert(!K16 || (FIXED && NB <= 65536), "16-bit keys need a single bucket set of <= 2^16");
  constexpr uint32_t SENTINEL = K16 ? 0u : FIXED ? NB : NW * NB;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    Fr s = scalars[i];
    if (mont) s = from_mont_fr29(s);
    uint32_t k[NW];
    uint32_t v[NW];
#pragma unroll
    for (int w = 0; w < NW; w++) {
      k[w] = SENTINEL;
      v[w] = K16 ? skip_val : (uint32_t)i;
    }
    for_each_digit<C>(s, [&](int w, uint32_t b, uint32_t sign) {
      if (FIXED) {
        k[w] = b;
        v[w] = (uint32_t)((size_t)w * stride + i) | (sign << 31);
      } else {
        k[w] = (uint32_t)w * NB + b;
        v[w] = (uint32_t)i | (sign << 31);
      }
    });
#pragma unroll
    for (int w = 0; w < NW; w++) {
      keys[(size_t)w * n + i] = (K)k[w];
      vals[(size_t)w * n + i] = v[w];
    }
  }
}

// ---- fixed-base bucketing (16-bit keys), replacing the library radix sort ------------
// Entries (one per scalar and window) are grouped by bucket in two counting passes, over
// the key's high byte and then its low byte, reduce-then-scan, with every counter in LDS
// or fully written (no look-back spinning, no fills):
//   1. msm_bin_hist_kernel    per tile of 512 scalars: the digits, and the histogram of
//                             the keys' high byte -> counts[hi][tile]
//   2. msm_bin_rowscan_kernel per high byte: exclusive scan over the tiles and the row
//                             total (consumers scan the 256 totals for the region starts)
//   3. msm_bin_scatter_kernel per tile: the digits again (32 B read per scalar instead of
//                             the 15 entries), ranked in LDS by high byte, then written
//                             out run by run (coalesced) into the high-byte regions: the
//                             value and the key's low byte
//   4. msm_lo_*_kernel        per high byte (split into segments, see below): low-byte histogram of its
//                             region, local scan -> the 256 bucket offsets, scatter
// Order inside a bucket is whatever the LDS atomics give: the accumulation adds the
// bucket's points in any order and the sum is the same point.
// 256- and 512-thread workgroups with modest LDS: under 5 proof lanes these kernels share
// the CUs with the accumulation's waves, and a 1024-thread or 95 KB-LDS workgroup waits
// for a whole CU to drain (measured: 5.3 ms average scatter launch in the pipeline)
static constexpr int kBinThreads = 256;
static constexpr int kBinPer = 2;                                  // scalars per thread and tile
static constexpr uint32_t kTileScalars = kBinThreads * kBinPer;    // 512
static constexpr int kLoThreads = 512;

// old = atomicAdd(&cnt[k], 1) for the lanes with `active`, where the lanes sharing the
// first active lane's key are served by ONE atomic of their count (each gets the old
// count plus its rank among them, an order the plain atomics could have given too).
// Same-address LDS atomics serialize: the Lagrange-basis commitments of 0/1-heavy witness
// columns put ~all of a region's entries in one bucket, and a workgroup walking 2^21 of
// them paid 64 cycles per wave-instruction (1.7 ms per launch, profiles/r3_single_lane_
// phases.txt). Every active lane of the wave calls it at the same point.
__device__ __forceinline__ uint32_t wave_agg_inc(uint32_t* cnt, uint32_t k, bool active) {
  const uint64_t act = __ballot(active);
  if (act == 0) return 0u;
  const int lead = __builtin_ctzll(act);
  const uint32_t k0 = __builtin_amdgcn_readlane(k, lead);
  const bool same = active && k == k0;
  const uint64_t m = __ballot(same);
  const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  uint32_t base = 0;
  if ((int)__lane_id() == lead) base = atomicAdd(&cnt[k0], (uint32_t)__popcll(m));
  base = __builtin_amdgcn_readlane(base, lead);
  if (same) return base + below;
  return active ? atomicAdd(&cnt[k], 1u) : 0u;
}

// the (key, value) of every window of scalar i; bit w of the result is set for the
// windows with a nonzero digit (zero digits make no entry: a scalar of b bits costs about
// b / C entries, which the Lagrange-basis commitments of small witness values rely on)
template <int C, int NW>
__device__ __forceinline__ uint32_t bin_entries(const Fr* __restrict__ scalars, size_t i, int mont, size_t stride,
                                                uint32_t (&kk)[NW], uint32_t (&vv)[NW]) {
  Fr s = scalars[i];
  if (mont) s = from_mont_fr29(s);
  uint32_t live = 0;
#pragma unroll
  for (int w = 0; w < NW; w++) {
    kk[w] = 0;
    vv[w] = 0;
  }
  for_each_digit<C>(s, [&](int w, uint32_t b, uint32_t sign) {
    kk[w] = b;
    vv[w] = (uint32_t)((size_t)w * stride + i) | (sign << 31);
    live |= 1u << w;
  });
  return live;
}

// bucket index bits below the high byte: 8 for c <= 17 (16-bit indices), c - 9 above
// (c = 20: 19-bit indices, 256 high-byte regions of 2048 buckets)
template <int C> struct BinKeys {
  static constexpr int LO = C - 9 > 8 ? C - 9 : 8;
  using Lo = typename std::conditional<LO <= 8, uint8_t, uint16_t>::type;      // low part, per entry
  using Full = typename std::conditional<C <= 17, uint16_t, uint32_t>::type;   // whole index, in LDS
};

template <int C>
__global__ void __launch_bounds__(kBinThreads)
msm_bin_hist_kernel(const Fr* __restrict__ scalars, size_t n, int mont, uint32_t* __restrict__ counts,
                    uint32_t ntiles) {
  constexpr int NW = (255 + C - 1) / C;
  constexpr int LO = BinKeys<C>::LO;
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kBinPer; j++) {
    const size_t i = (size_t)blockIdx.x * kTileScalars + (size_t)j * kBinThreads + threadIdx.x;
    if (i < n) {
      uint32_t kk[NW], vv[NW];
      const uint32_t live = bin_entries<C, NW>(scalars, i, mont, 0, kk, vv);
#pragma unroll
      for (int w = 0; w < NW; w++)
        if ((live >> w) & 1u) atomicAdd(&h[kk[w] >> LO], 1u);
    }
  }
  __syncthreads();
  counts[(size_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

// wave64 inclusive scan
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t u = __shfl_up(v, off, 64);
    if (lane >= off) v += u;
  }
  return v;
}

// exclusive scan of v over the first 256 threads of the workgroup (blockDim >= 256; every
// thread calls it): returns the thread's exclusive prefix (threads >= 256: 0) and the
// total of the 256 values
__device__ __forceinline__ uint32_t scan256_excl(uint32_t v, uint32_t* wsum4, uint32_t& total) {
  const uint32_t inc = wave_incl_scan(threadIdx.x < 256 ? v : 0u);
  if (threadIdx.x < 256 && (threadIdx.x & 63) == 63) wsum4[threadIdx.x >> 6] = inc;
  __syncthreads();
  uint32_t off = 0;
  for (int w = 0; w < (int)(threadIdx.x >> 6) && w < 4; w++) off += wsum4[w];
  total = wsum4[0] + wsum4[1] + wsum4[2] + wsum4[3];
  __syncthreads();
  return threadIdx.x < 256 ? off + inc - v : 0u;
}

// one workgroup (256 threads) per high byte hb: exclusive scan of counts[hb][0..ntiles) in
// place (coalesced 256-wide chunks with a running carry), row total -> tail[hb]
__global__ void __launch_bounds__(256)
msm_bin_rowscan_kernel(uint32_t* __restrict__ counts, uint32_t ntiles, uint32_t* __restrict__ tail) {
  __shared__ uint32_t wsum[4];
  uint32_t* row = counts + (size_t)blockIdx.x * ntiles;
  uint32_t carry = 0;
  for (uint32_t c0 = 0; c0 < ntiles; c0 += 256) {
    const uint32_t t = c0 + threadIdx.x;
    const uint32_t v = t < ntiles ? row[t] : 0u;
    uint32_t tot;
    const uint32_t ex = scan256_excl(v, wsum, tot);
    if (t < ntiles) row[t] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) tail[blockIdx.x] = carry;
}

template <int C>
__global__ void __launch_bounds__(kBinThreads)
msm_bin_scatter_kernel(const Fr* __restrict__ scalars, size_t n, int mont, size_t stride,
                       const uint32_t* __restrict__ counts, uint32_t ntiles, typename BinKeys<C>::Lo* __restrict__ lo2,
                       uint32_t* __restrict__ vals2) {
  constexpr int NW = (255 + C - 1) / C;
  constexpr int TE = kTileScalars * NW;  // entries per tile, at most
  constexpr int LO = BinKeys<C>::LO;
  __shared__ uint32_t lcount[256], lstart[256], gbase[256];
  __shared__ uint32_t lval[TE];
  __shared__ typename BinKeys<C>::Full lkey[TE];
  __shared__ uint32_t wsum[4];
  const uint32_t* tail = counts + (size_t)256 * ntiles;  // row totals
  {
    uint32_t tot;
    const uint32_t st = scan256_excl(tail[threadIdx.x], wsum, tot);  // start of region threadIdx.x
    gbase[threadIdx.x] = st + counts[(size_t)threadIdx.x * ntiles + blockIdx.x];
    lcount[threadIdx.x] = 0;
  }
  __syncthreads();
  uint32_t kk[kBinPer][NW], vv[kBinPer][NW], rk[kBinPer][NW], live[kBinPer];
#pragma unroll
  for (int j = 0; j < kBinPer; j++) {
    const size_t i = (size_t)blockIdx.x * kTileScalars + (size_t)j * kBinThreads + threadIdx.x;
    live[j] = 0;
    if (i < n) {
      live[j] = bin_entries<C, NW>(scalars, i, mont, stride, kk[j], vv[j]);
#pragma unroll
      for (int w = 0; w < NW; w++)
        if ((live[j] >> w) & 1u) rk[j][w] = atomicAdd(&lcount[kk[j][w] >> LO], 1u);
    }
  }
  __syncthreads();
  uint32_t total;
  {  // exclusive scan of the tile's 256 high-byte counts; total = the tile's entries
    lstart[threadIdx.x] = scan256_excl(lcount[threadIdx.x], wsum, total);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kBinPer; j++) {
#pragma unroll
    for (int w = 0; w < NW; w++) {
      if ((live[j] >> w) & 1u) {
        const uint32_t q = lstart[kk[j][w] >> LO] + rk[j][w];
        lkey[q] = (typename BinKeys<C>::Full)kk[j][w];
        lval[q] = vv[j][w];
      }
    }
  }
  __syncthreads();
  for (uint32_t q = threadIdx.x; q < total; q += kBinThreads) {  // runs of one high byte: coalesced
    const uint32_t key = lkey[q], hb = key >> LO;
    const uint32_t pos = gbase[hb] + (q - lstart[hb]);
    lo2[pos] = (typename BinKeys<C>::Lo)(key & ((1u << LO) - 1u));
    vals2[pos] = lval[q];
  }
}

// exclusive scan in place of a[0..count) by an NT-thread workgroup (every thread calls it,
// after a barrier that completes a[]); returns the total. wsum: NT / 64 words of LDS.
template <int NT>
__device__ __forceinline__ uint32_t block_scan_excl(uint32_t* a, uint32_t count, uint32_t* wsum) {
  const uint32_t per = (count + NT - 1) / NT;
  const uint32_t b = threadIdx.x * per;
  uint32_t loc = 0;
  for (uint32_t i = 0; i < per; i++)
    if (b + i < count) loc += a[b + i];
  const uint32_t inc = wave_incl_scan(loc);
  if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = inc;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; w++) {
    if (w < (int)(threadIdx.x >> 6)) off += wsum[w];
    tot += wsum[w];
  }
  uint32_t run = off + inc - loc;
  for (uint32_t i = 0; i < per; i++)
    if (b + i < count) {
      const uint32_t v = a[b + i];
      a[b + i] = run;
      run += v;
    }
  __syncthreads();
  return tot;
}

// Step 4 runs over work items of at most kLoSeg entries (the segments of the high-byte
// regions, in region order), so a region holding most of the entries (the Lagrange-basis
// commitments of 0/1-heavy witness columns: ~all 2^21 entries in bucket 0's region) is
// spread over many workgroups instead of one (1.2 ms for that region's single workgroup
// even with aggregated atomics; 0.1 ms for random scalars):
//   a. msm_lo_count_kernel   per item: low-index histogram of its segment -> segoff[item][.]
//   b. msm_lo_scan_kernel    per region: exclusive scan over its items per bucket, the
//                            bucket offsets (scan over the buckets), segoff += bucket offset
//   c. msm_lo_scatter_kernel per item: ranked in LDS chunk by chunk, written run by run
static constexpr uint32_t kLoSeg = 32768;
static constexpr uint32_t kLoU = 8;  // entries per thread and chunk

// kAgg (NZCB_LO_AGG=1): the lanes sharing a key served by one LDS atomic (wave_agg_inc);
// by default plain atomics: with regions cut into kLoSeg segments a hot bucket's
// same-address conflicts cost ~15 us per workgroup, and the aggregation's ~10 extra
// instructions per entry ran on every entry of every MSM
template <bool kAgg>
__device__ __forceinline__ uint32_t lo_inc(uint32_t* cnt, uint32_t k, bool active) {
  if (kAgg) return wave_agg_inc(cnt, k, active);
  return active ? atomicAdd(&cnt[k], 1u) : 0u;
}

// rs[r] = first entry of high-byte region r, rf[r] = its first work item (rf[256] = all
// items). Every thread of the workgroup calls it (barriers inside).
__device__ __forceinline__ void lo_regions(const uint32_t* __restrict__ tail, uint32_t* wsum, uint32_t* rs,
                                           uint32_t* rf) {
  const uint32_t t = threadIdx.x;
  const uint32_t cnt = t < 256 ? tail[t] : 0u;
  uint32_t tot, nitems;
  const uint32_t st = scan256_excl(cnt, wsum, tot);
  const uint32_t f = scan256_excl((cnt + kLoSeg - 1) / kLoSeg, wsum, nitems);
  if (t < 256) {
    rs[t] = st;
    rf[t] = f;
  }
  if (t == 0) rf[256] = nitems;
  __syncthreads();
}

// the region of work item `item` (< rf[256]): the largest r with rf[r] <= item
__device__ __forceinline__ uint32_t lo_region_of(const uint32_t* rf, uint32_t item) {
  uint32_t lo = 0, hi = 256;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (rf[mid] <= item) lo = mid; else hi = mid;
  }
  return lo;
}

template <int LO, bool kAgg>
__global__ void __launch_bounds__(kLoThreads)
msm_lo_count_kernel(const typename std::conditional<LO <= 8, uint8_t, uint16_t>::type* __restrict__ lo2,
                    const uint32_t* __restrict__ counts, uint32_t ntiles, uint32_t* __restrict__ segoff) {
  constexpr uint32_t NL = 1u << LO;
  __shared__ uint32_t h[NL], wsum[kLoThreads / 64], rs[256], rf[257];
  lo_regions(counts + (size_t)256 * ntiles, wsum, rs, rf);
  const uint32_t item = blockIdx.x;
  if (item >= rf[256]) return;
  const uint32_t r = lo_region_of(rf, item);
  const uint32_t* tail = counts + (size_t)256 * ntiles;
  const uint32_t s = rs[r] + (item - rf[r]) * kLoSeg;
  const uint32_t e = min(rs[r] + tail[r], s + kLoSeg);
  for (uint32_t i = threadIdx.x; i < NL; i += kLoThreads) h[i] = 0;
  __syncthreads();
  for (uint32_t p0 = s; p0 < e; p0 += kLoU * kLoThreads) {
    uint32_t k8[kLoU];
#pragma unroll
    for (uint32_t u = 0; u < kLoU; u++) {  // independent loads in flight before the atomics
      const uint32_t q = p0 + u * kLoThreads + threadIdx.x;
      k8[u] = q < e ? (uint32_t)lo2[q] : NL;
    }
#pragma unroll
    for (uint32_t u = 0; u < kLoU; u++) lo_inc<kAgg>(h, k8[u], k8[u] < NL);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < NL; i += kLoThreads) segoff[(size_t)item * NL + i] = h[i];
}

template <int LO>
__global__ void __launch_bounds__(kLoThreads)
msm_lo_scan_kernel(const uint32_t* __restrict__ counts, uint32_t ntiles, uint32_t* __restrict__ segoff,
                   uint32_t nkeys, uint32_t* __restrict__ offsets, uint32_t* __restrict__ large) {
  constexpr uint32_t NL = 1u << LO;
  __shared__ uint32_t h[NL], wsum[kLoThreads / 64], rs[256], rf[257];
  const uint32_t* tail = counts + (size_t)256 * ntiles;
  lo_regions(tail, wsum, rs, rf);
  const uint32_t hb = blockIdx.x;
  const uint32_t f0 = rf[hb], ns = rf[hb + 1] - f0, s = rs[hb];
  for (uint32_t i = threadIdx.x; i < NL; i += kLoThreads) {  // bucket i: its items' counts -> exclusive
    uint32_t run = 0;
    for (uint32_t g = 0; g < ns; g++) {
      uint32_t* c = segoff + (size_t)(f0 + g) * NL + i;
      const uint32_t v = *c;
      *c = run;
      run += v;
    }
    h[i] = run;
  }
  __syncthreads();
  block_scan_excl<kLoThreads>(h, NL, wsum);  // bucket totals -> offsets in the region
  for (uint32_t i = threadIdx.x; i < NL; i += kLoThreads) {
    const uint32_t base = s + h[i];
    const uint32_t key = (hb << LO) | i;
    if (key < nkeys) offsets[key] = base;
    for (uint32_t g = 0; g < ns; g++) segoff[(size_t)(f0 + g) * NL + i] += base;
  }
  if (hb == 255 && threadIdx.x == 0) offsets[nkeys] = s + tail[255];  // entries in all
  if (hb == 0 && threadIdx.x == 0) large[0] = 0;                     // the finalize's count of long runs
}

template <int LO, bool kAgg>
__global__ void __launch_bounds__(kLoThreads)
msm_lo_scatter_kernel(const typename std::conditional<LO <= 8, uint8_t, uint16_t>::type* __restrict__ lo2,
                      const uint32_t* __restrict__ vals2, const uint32_t* __restrict__ counts, uint32_t ntiles,
                      const uint32_t* __restrict__ segoff, uint32_t* __restrict__ sorted) {
  using Lo = typename std::conditional<LO <= 8, uint8_t, uint16_t>::type;
  constexpr uint32_t NL = 1u << LO;
  __shared__ uint32_t h[NL], lcnt[NL], lst[NL];
  __shared__ uint32_t wsum[kLoThreads / 64], rs[256], rf[257];
  __shared__ uint32_t lv[kLoU * kLoThreads];
  __shared__ Lo lk[kLoU * kLoThreads];
  lo_regions(counts + (size_t)256 * ntiles, wsum, rs, rf);
  const uint32_t item = blockIdx.x;
  if (item >= rf[256]) return;
  const uint32_t r = lo_region_of(rf, item);
  const uint32_t* tail = counts + (size_t)256 * ntiles;
  const uint32_t s = rs[r] + (item - rf[r]) * kLoSeg;
  const uint32_t e = min(rs[r] + tail[r], s + kLoSeg);
  for (uint32_t i = threadIdx.x; i < NL; i += kLoThreads) h[i] = segoff[(size_t)item * NL + i];
  for (uint32_t p0 = s; p0 < e; p0 += kLoU * kLoThreads) {
    uint32_t k8[kLoU], v8[kLoU], r8[kLoU];
    for (uint32_t i = threadIdx.x; i < NL; i += kLoThreads) lcnt[i] = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < kLoU; u++) {
      const uint32_t q = p0 + u * kLoThreads + threadIdx.x;
      k8[u] = q < e ? (uint32_t)lo2[q] : NL;
      v8[u] = q < e ? vals2[q] : 0u;
    }
#pragma unroll
    for (uint32_t u = 0; u < kLoU; u++) r8[u] = lo_inc<kAgg>(lcnt, k8[u], k8[u] < NL);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < NL; i += kLoThreads) lst[i] = lcnt[i];
    __syncthreads();
    block_scan_excl<kLoThreads>(lst, NL, wsum);
#pragma unroll
    for (uint32_t u = 0; u < kLoU; u++)
      if (k8[u] < NL) {
        const uint32_t q = lst[k8[u]] + r8[u];
        lk[q] = (Lo)k8[u];
        lv[q] = v8[u];
      }
    __syncthreads();
    const uint32_t cnt = e - p0 < kLoU * kLoThreads ? e - p0 : kLoU * kLoThreads;
    for (uint32_t q = threadIdx.x; q < cnt; q += kLoThreads) {  // runs of one bucket: coalesced
      const uint32_t k = lk[q];
      sorted[h[k] + (q - lst[k])] = lv[q];
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < NL; i += kLoThreads) h[i] += lcnt[i];
  }
}

// Round-2 step 4 (NZCB_LO_SPLIT=0, A/B runs): one workgroup per high-byte region.
template <int LO>
__global__ void __launch_bounds__(kLoThreads)
msm_bucket_lo_kernel(const typename std::conditional<LO <= 8, uint8_t, uint16_t>::type* __restrict__ lo2,
                     const uint32_t* __restrict__ vals2, const uint32_t* __restrict__ counts, uint32_t ntiles,
                     uint32_t nkeys, uint32_t* __restrict__ offsets, uint32_t* __restrict__ sorted,
                     uint32_t* __restrict__ large) {
  using Lo = typename std::conditional<LO <= 8, uint8_t, uint16_t>::type;
  constexpr uint32_t NL = 1u << LO;  // buckets per high-byte region
  constexpr uint32_t U = 8;
  __shared__ uint32_t h[NL], lcnt[NL], lst[NL];
  __shared__ uint32_t wsum[kLoThreads / 64], reg[1];
  __shared__ uint32_t lv[U * kLoThreads];
  __shared__ Lo lk[U * kLoThreads];
  const uint32_t hb = blockIdx.x;
  const uint32_t* tail = counts + (size_t)256 * ntiles;  // row totals
  {
    uint32_t tot;
    const uint32_t st = scan256_excl(threadIdx.x < 256 ? tail[threadIdx.x] : 0u, wsum, tot);
    if (threadIdx.x == hb) reg[0] = st;  // this region's start
  }
  for (uint32_t i = threadIdx.x; i < NL; i += kLoThreads) h[i] = 0;
  __syncthreads();
  const uint32_t s = reg[0];
  const uint32_t e = s + tail[hb];
  // 8 independent loads in flight per thread before their atomics (the loop is
  // latency-bound otherwise: one workgroup per CU walks ~entries/256 entries)
  for (uint32_t p0 = s; p0 < e; p0 += U * kLoThreads) {
    uint32_t k8[U];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint32_t p = p0 + u * kLoThreads + threadIdx.x;
      k8[u] = p < e ? (uint32_t)lo2[p] : NL;
    }
#pragma unroll
    for (uint32_t u = 0; u < U; u++)
      if (k8[u] < NL) atomicAdd(&h[k8[u]], 1u);
  }
  __syncthreads();
  block_scan_excl<kLoThreads>(h, NL, wsum);  // low-index counts -> bucket offsets in the region
  for (uint32_t i = threadIdx.x; i < NL; i += kLoThreads) {
    h[i] += s;
    const uint32_t key = (hb << LO) | i;
    if (key < nkeys) offsets[key] = h[i];
  }
  if (hb == 255 && threadIdx.x == 0) offsets[nkeys] = e;  // entries in all: the last region's end
  if (hb == 0 && threadIdx.x == 0) large[0] = 0;          // the finalize's count of long bucket runs
  __syncthreads();
  // scatter in chunks of U * kLoThreads entries, each ranked by low index in LDS first and
  // written out run by run (coalesced)
  for (uint32_t p0 = s; p0 < e; p0 += U * kLoThreads) {
    uint32_t k8[U], v8[U], r8[U];
    for (uint32_t i = threadIdx.x; i < NL; i += kLoThreads) lcnt[i] = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint32_t p = p0 + u * kLoThreads + threadIdx.x;
      k8[u] = p < e ? (uint32_t)lo2[p] : NL;
      v8[u] = p < e ? vals2[p] : 0u;
    }
#pragma unroll
    for (uint32_t u = 0; u < U; u++)
      if (k8[u] < NL) r8[u] = atomicAdd(&lcnt[k8[u]], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < NL; i += kLoThreads) lst[i] = lcnt[i];
    __syncthreads();
    block_scan_excl<kLoThreads>(lst, NL, wsum);
#pragma unroll
    for (uint32_t u = 0; u < U; u++)
      if (k8[u] < NL) {
        const uint32_t q = lst[k8[u]] + r8[u];
        lk[q] = (Lo)k8[u];
        lv[q] = v8[u];
      }
    __syncthreads();
    const uint32_t cnt = e - p0 < U * kLoThreads ? e - p0 : U * kLoThreads;
    for (uint32_t q = threadIdx.x; q < cnt; q += kLoThreads) {
      const uint32_t k = lk[q];
      sorted[h[k] + (q - lst[k])] = lv[q];
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < NL; i += kLoThreads) h[i] += lcnt[i];
  }
}

static bool use_library_sort() {
  static const bool v = [] {
    const char* e = std::getenv("NZCB_ROCPRIM_SORT");
    return e && std::atoi(e) != 0;
  }();
  return v;
}

// offsets[k] = first position of a key >= k in the sorted key array (k = 0..nkeys)
template <class K>
__global__ void __launch_bounds__(kMsmThreads)
msm_offsets_kernel(const K* __restrict__ skeys, size_t m, uint32_t nkeys, uint32_t* __restrict__ offsets) {
  size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k > nkeys) return;
  size_t lo = 0, hi = m;
  while (lo < hi) {
    size_t mid = (lo + hi) >> 1;
    if (skeys[mid] < k) lo = mid + 1; else hi = mid;
  }
  offsets[k] = (uint32_t)lo;
}

// largest k in [0, nkeys) with offsets[k] <= pos  (offsets[nkeys] > pos)
__device__ __forceinline__ uint32_t find_key(const uint32_t* __restrict__ offsets, uint32_t nkeys, uint32_t pos) {
  uint32_t lo = 0, hi = nkeys;
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (offsets[mid] <= pos) lo = mid; else hi = mid;
  }
  return lo;
}

__global__ void __launch_bounds__(kMsmThreads)
msm_accumulate_kernel(uint32_t chunk, const G1Affine* __restrict__ bases, const uint32_t* __restrict__ sorted,
                      const uint32_t* __restrict__ offsets, uint32_t nkeys, size_t nthreads,
                      G1xyzz* __restrict__ buckets, G1xyzz* __restrict__ carry_own,
                      G1xyzz* __restrict__ carry_cont) {
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nthreads) return;
  const uint32_t M = offsets[nkeys];
  const uint32_t s = (uint32_t)t * chunk;
  if (s >= M) return;
  const uint32_t e = (s + chunk < M) ? s + chunk : M;
  uint32_t k = find_key(offsets, nkeys, s);
  uint32_t kstart = offsets[k], kend = offsets[k + 1];
  G1xyzz acc = G1xyzz::inf();
  for (uint32_t pos = s; pos < e;) {
    const uint32_t ent = sorted[pos];
    const G1Affine P = bases[ent & 0x7fffffffu];
    if (!P.is_inf()) {
      Fq y = (ent >> 31) ? neg(P.y) : P.y;
      acc = xyzz_add_affine(acc, P.x, y);
    }
    pos++;
    if (pos == kend || pos == e) {
      const bool starts = kstart >= s;
      const bool ends = kend <= e;
      if (starts && ends) buckets[k] = acc;
      else if (!starts) carry_cont[t] = acc;
      else carry_own[t] = acc;
      acc = G1xyzz::inf();
      if (pos < e) {
        k = find_key(offsets, nkeys, pos);
        kstart = offsets[k];
        kend = offsets[k + 1];
      }
    }
  }
}

// Fixed-base schedule: the same chunked accumulation in the redundant radix 2^29
// (csrc/f29.h) on table bases stored as Montgomery-261 values. Results are stored
// unconverted (a store per bucket run costs a few instructions; the 4 products of the
// conversion would run for the whole wave whenever any lane ends a run, i.e. on most
// iterations) and the finalize kernel converts them to the Montgomery-256 layout.
static __device__ __forceinline__ void mdbl29_rare(const F29& x, const F29& y, Xyzz29* out) { *out = mdbl29(x, y); }

__device__ __forceinline__ G1xyzz load_point(const G1xyzz& p) { return p; }
__device__ __forceinline__ G1xyzz load_point(const Xyzz29& a) {
  uint32_t z = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) z |= a.ZZ.v[i];
  if (!z) return G1xyzz::inf();
  G1xyzz r;
  r.X = to_fq256(a.X);
  r.Y = to_fq256(a.Y);
  r.ZZ = to_fq256(a.ZZ);
  r.ZZZ = to_fq256(a.ZZZ);
  return r;
}

// kDirect: entries are the pairing rounds' affine sums (msm_pair29_kernel), read in
// place (position = entry), instead of signed table indices in `sorted`.
// kLdsIdx (chunk == kChunk): the workgroup's kMsmThreads x kChunk slice of `sorted` is
// staged into LDS by coalesced loads before the additions. Read from HBM one index per
// addition, each lane's chunk 192 B from its neighbour's, the index lines were evicted
// between uses by the table gathers and fetched again (~1 GB of the 3.3 GB a launch
// moved, profiles/r2_fetch_calibration.txt); a gather-only probe over the same stream
// ran 1.08 ms with HBM indices and 0.65 ms with LDS ones (tools/table_probe.hip).
// 49 KB per workgroup: three workgroups (12 waves, the 3 waves per SIMD the kernel is
// compiled for) fit the CU's 160 KB.
static constexpr uint32_t kLdsStride = kMsmThreads + 1;  // slot-major rows, +1: conflict-free fill
// kPair: the addition's independent products in interleaved pairs (mul29x2 / sqr29x2:
// U2 | S2, PP | RR, PPP | Q, ZZ3 | ZZZ3), two v_mad_u64_u32 chains per asm statement
// kAff: the addition right after a run's first entry (acc = (x, y, 1, 1), every lane of a
// wave at once at step 1 of the chunks) skips the products by ZZ1 = ZZZ1 = 1: U2 = x, S2 = y,
// ZZ3 = PP, ZZZ3 = PPP (a wave-uniform branch around two product pairs, one addition site)
template <int WAVES, bool kDirect = false, bool kLdsIdx = false, bool kPair = false, bool kAff = false>
__global__ void __launch_bounds__(kMsmThreads) __attribute__((amdgpu_waves_per_eu(WAVES, 8)))
msm_accumulate29_kernel(uint32_t chunk, const G1Affine* __restrict__ bases, const uint32_t* __restrict__ sorted,
                        const uint32_t* __restrict__ offsets, uint32_t nkeys, size_t nthreads,
                        Xyzz29* __restrict__ buckets, Xyzz29* __restrict__ carry_own,
                        Xyzz29* __restrict__ carry_cont) {
  __shared__ uint32_t sidx[kLdsIdx ? kChunk * kLdsStride : 1];
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t M = offsets[nkeys];
  if (kLdsIdx) {  // every thread of the workgroup takes part before any exits
    const uint32_t wg0 = (uint32_t)blockIdx.x * kMsmThreads * kChunk;
    for (uint32_t j = threadIdx.x; j < kMsmThreads * kChunk; j += kMsmThreads) {
      const uint32_t thr = j / kChunk, slot = j - thr * kChunk;
      sidx[slot * kLdsStride + thr] = wg0 + j < M ? sorted[wg0 + j] : 0u;
    }
    __syncthreads();
  }
  if (t >= nthreads) return;
  const uint32_t s = (uint32_t)t * chunk;
  if (s >= M) return;
  const uint32_t e = (s + chunk < M) ? s + chunk : M;
  // index of stream position q (kLdsIdx: q - s is this thread's slot)
  auto index_at = [&](uint32_t q) -> uint32_t {
    return kLdsIdx ? sidx[(q - s) * kLdsStride + threadIdx.x] : sorted[q];
  };
  uint32_t k = find_key(offsets, nkeys, s);
  uint32_t kstart = offsets[k], kend = offsets[k + 1];
  Xyzz29 acc;
  bool inf = true, aff = false;
  // software pipeline: the next entry's table point is loaded before this entry's
  // addition, so the gather's latency hides behind ~8k cycles of arithmetic, and the
  // entry after it is read one step earlier still, so that gather's address is in a
  // register when it is issued (no wait on the index load inside an iteration)
  uint32_t ent = kDirect ? 0u : index_at(s);
  G1Affine P = bases[kDirect ? s : ent & 0x7fffffffu];
  uint32_t ent_n = (!kDirect && s + 1 < e) ? index_at(s + 1) : 0u;
  for (uint32_t pos = s; pos < e;) {
    G1Affine Pn;
    uint32_t ent_nn = 0;
    if (pos + 1 < e) Pn = bases[kDirect ? pos + 1 : ent_n & 0x7fffffffu];
    if (!kDirect && pos + 2 < e) ent_nn = index_at(pos + 2);
    if (!P.is_inf()) {
      const F29 x = split29(P.x);
      F29 y = split29(P.y);
      if (ent >> 31) y = neg29_nn(y);  // 2p - y, limbs < 2^30: only S2's product reads it
      if (inf) {
        norm29(y);
        acc.X = x;
        acc.Y = y;
        acc.ZZ = f29_const(Fq29::ONE);
        acc.ZZZ = f29_const(Fq29::ONE);
        inf = false;
        aff = kAff;
      } else if (kPair) {
        // madd-2008-s as above, products paired
        F29 U2, S2, PP, RR;
        if (kAff && aff) {  // x ZZ1 = x, y ZZZ1 = y (ONE is the Montgomery-261 1)
          U2 = x;
          S2 = y;  // 2p - y for a negated digit: limbs < 2^30, sub29 normalizes R
        } else {
          mul29x2<Fq29>(x, acc.ZZ, y, acc.ZZZ, U2, S2);
        }
        const F29 Pd = sub29(U2, acc.X, Fq29::K8);   // < 10p
        const F29 R = sub29(S2, acc.Y, Fq29::K4);    // < 6p
        sqr29x2(Pd, R, PP, RR);
        if (is0p29_fast(PP)) {  // same abscissa: doubling (equal points) or infinity (opposite)
          if (is0p29(RR)) {
            norm29(y);
            mdbl29_rare(x, y, &acc);
          } else {
            inf = true;
          }
        } else {
          F29 PPP, Q, ZZ3, ZZZ3;
          mul29x2<Fq29>(Pd, PP, acc.X, PP, PPP, Q);
          const F29 X3 = sub2x29(RR, PPP, Q);  // RR + 6p - PPP - 2Q < 8p
          if (kAff && aff) {
            ZZ3 = PP;
            ZZZ3 = PPP;
          } else {
            mul29x2<Fq29>(acc.ZZ, PP, acc.ZZZ, PPP, ZZ3, ZZZ3);
          }
          acc.Y = mul2sum29(R, sub29_nn(Q, X3, Fq29W::K10), neg4p29_nn(acc.Y), PPP);
          acc.ZZ = ZZ3;
          acc.ZZZ = ZZZ3;
          acc.X = X3;
        }
        aff = false;
      } else {
        // madd-2008-s (XYZZ + affine): 8 products + 2 squares
        const F29 U2 = mul29(x, acc.ZZ);
        const F29 S2 = mul29(y, acc.ZZZ);
        const F29 Pd = sub29(U2, acc.X, Fq29::K8);   // < 10p
        const F29 R = sub29(S2, acc.Y, Fq29::K4);    // < 6p
        const F29 PP = sqr29(Pd);
        if (is0p29_fast(PP)) {  // same abscissa: doubling (equal points) or infinity (opposite)
          if (is0p29(sqr29(R))) {
            norm29(y);
            mdbl29_rare(x, y, &acc);
          } else {
            inf = true;
          }
        } else {  // x, y are dead from here on (lower register pressure in the common path)
          const F29 PPP = mul29(Pd, PP);
          const F29 Q = mul29(acc.X, PP);
          const F29 RR = sqr29(R);
          const F29 X3 = sub2x29(RR, PPP, Q);  // RR + 6p - PPP - 2Q < 8p
          acc.ZZ = mul29(acc.ZZ, PP);
          // Y3 = R (Q - X3) + (4p - Y1) PPP, one reduction: (6p 12p + 4p 2p) / 2^261 + p < 2p;
          // Q - X3 + 10p (limbs < 2^30.6) and 4p - Y1 (limbs < 2^30) stay unnormalized
          acc.Y = mul2sum29(R, sub29_nn(Q, X3, Fq29W::K10), neg4p29_nn(acc.Y), PPP);
          acc.ZZZ = mul29(acc.ZZZ, PPP);
          acc.X = X3;
        }
      }
    }
    pos++;
    if (pos == kend || pos == e) {
      const bool starts = kstart >= s;
      const bool ends = kend <= e;
      Xyzz29 out = acc;
      if (inf)
#pragma unroll
        for (int i = 0; i < 9; i++) out.ZZ.v[i] = 0;
      if (starts && ends) buckets[k] = out;
      else if (!starts) carry_cont[t] = out;
      else carry_own[t] = out;
      inf = true;
      // next non-empty bucket: a linear walk (one load per bucket; runs average
      // entries / nkeys ~ 480 at 2^21, so a chunk crosses at most a few boundaries)
      while (pos < e && kend <= pos) {
        k++;
        kstart = kend;
        kend = offsets[k + 1];
      }
    }
    ent = ent_n;
    ent_n = ent_nn;
    P = Pn;
  }
}

// 4 waves per SIMD (NZCB_ACC_DMA=1, A/B runs). At 4 waves (<= 128 VGPRs) the register-
// prefetched next point of msm_accumulate29_kernel spilled to scratch; here the next
// entry's table point goes HBM -> LDS by global_load_lds_dwordx4 (four 16-byte quarters
// per lane, no VGPRs held while it is in flight) and is read back at the top of the next
// iteration. The indices are staged kDmaGroup slots at a time (two barriers per group; every
// thread of the workgroup runs the same kChunk iterations, finished or not), so one
// workgroup needs 16 x 257 x 4 B of indices + 256 x 64 B of points = 32.4 KB and four fit
// a CU (16 waves). Same additions, same results as the 3-wave kernel.
static constexpr uint32_t kDmaGroup = 16;
static_assert(kChunk % kDmaGroup == 0, "index groups tile the chunk");

// x, y die after the first product pair: the rare doubling reloads its point from the
// table (`pt`, `neg`) instead of keeping 18 VGPRs live through the whole addition
__device__ __forceinline__ void acc_madd29(Xyzz29& acc, bool& inf, const F29& x, F29 y,
                                           const G1Affine* __restrict__ pt, bool neg) {
  if (inf) {
    norm29(y);
    acc.X = x;
    acc.Y = y;
    acc.ZZ = f29_const(Fq29::ONE);
    acc.ZZZ = f29_const(Fq29::ONE);
    inf = false;
    return;
  }
  // madd-2008-s with the products paired (as msm_accumulate29_kernel kPair)
  F29 U2, S2, PP, RR;
  mul29x2<Fq29>(x, acc.ZZ, y, acc.ZZZ, U2, S2);
  const F29 Pd = sub29(U2, acc.X, Fq29::K8);   // < 10p
  const F29 R = sub29(S2, acc.Y, Fq29::K4);    // < 6p
  sqr29x2(Pd, R, PP, RR);
  if (is0p29_fast(PP)) {  // same abscissa: doubling (equal points) or infinity (opposite)
    if (is0p29(RR)) {
      const G1Affine P = *pt;
      const F29 x2 = split29(P.x);
      F29 y2 = split29(P.y);
      if (neg) y2 = neg29_nn(y2);
      norm29(y2);
      mdbl29_rare(x2, y2, &acc);
    } else {
      inf = true;
    }
    return;
  }
  F29 PPP, Q, ZZ3, ZZZ3;
  mul29x2<Fq29>(Pd, PP, acc.X, PP, PPP, Q);
  const F29 X3 = sub2x29(RR, PPP, Q);  // RR + 6p - PPP - 2Q < 8p
  mul29x2<Fq29>(acc.ZZ, PP, acc.ZZZ, PPP, ZZ3, ZZZ3);
  acc.Y = mul2sum29(R, sub29_nn(Q, X3, Fq29W::K10), neg4p29_nn(acc.Y), PPP);
  acc.ZZ = ZZ3;
  acc.ZZZ = ZZZ3;
  acc.X = X3;
}

__global__ void __launch_bounds__(kMsmThreads) __attribute__((amdgpu_waves_per_eu(4, 8)))
msm_accumulate29_dma_kernel(const G1Affine* __restrict__ bases, const uint32_t* __restrict__ sorted,
                            const uint32_t* __restrict__ offsets, uint32_t nkeys, size_t nthreads,
                            Xyzz29* __restrict__ buckets, Xyzz29* __restrict__ carry_own,
                            Xyzz29* __restrict__ carry_cont) {
  __shared__ uint32_t sidx[kDmaGroup * kLdsStride];
  __shared__ uint4 spt[4 * kMsmThreads];  // [wave][quarter][lane], 16 B each
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t M = offsets[nkeys];
  const uint32_t wg0 = (uint32_t)blockIdx.x * kMsmThreads * kChunk;
  const uint32_t s = (uint32_t)t * kChunk;
  const bool live = t < nthreads && s < M;
  const uint32_t e = live ? (s + kChunk < M ? s + kChunk : M) : s;
  const uint32_t lane = threadIdx.x & 63;
  uint4* wpt = spt + (threadIdx.x >> 6) * 256;
  auto stage = [&](uint32_t g) {  // slots [g kDmaGroup, (g + 1) kDmaGroup) of every thread's chunk
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < kMsmThreads * kDmaGroup; j += kMsmThreads) {
      const uint32_t thr = j / kDmaGroup, slot = j - thr * kDmaGroup;
      const uint32_t q = wg0 + thr * kChunk + g * kDmaGroup + slot;
      sidx[slot * kLdsStride + thr] = q < M ? sorted[q] : 0u;
    }
    __syncthreads();
  };
  auto dma = [&](uint32_t ent) {  // table point of `ent` -> this lane's four LDS quarters
    const uint4* src = (const uint4*)(bases + (ent & 0x7fffffffu));
#pragma unroll
    for (int qq = 0; qq < 4; qq++)
      __builtin_amdgcn_global_load_lds((const void*)(src + qq),
                                       (__attribute__((address_space(3))) void*)(wpt + qq * 64), 16, 0, 0);
  };
  stage(0);
  uint32_t k = 0, kstart = 0, kend = 0;
  if (live) {
    k = find_key(offsets, nkeys, s);
    kstart = offsets[k];
    kend = offsets[k + 1];
  }
  uint32_t ent = sidx[threadIdx.x];
  dma(ent);
  Xyzz29 acc;
  bool inf = true;
  for (uint32_t j = 0; j < kChunk; j++) {
    const uint32_t pos = s + j;
    const uint4 q0 = wpt[lane], q1 = wpt[64 + lane], q2 = wpt[128 + lane], q3 = wpt[192 + lane];
    G1Affine P;
    P.x.v[0] = q0.x; P.x.v[1] = q0.y; P.x.v[2] = q0.z; P.x.v[3] = q0.w;
    P.x.v[4] = q1.x; P.x.v[5] = q1.y; P.x.v[6] = q1.z; P.x.v[7] = q1.w;
    P.y.v[0] = q2.x; P.y.v[1] = q2.y; P.y.v[2] = q2.z; P.y.v[3] = q2.w;
    P.y.v[4] = q3.x; P.y.v[5] = q3.y; P.y.v[6] = q3.z; P.y.v[7] = q3.w;
    const bool use = pos < e && !P.is_inf();
    const uint32_t ent_cur = ent;
    const F29 x = split29(P.x);
    F29 y = split29(P.y);
    if (ent >> 31) y = neg29_nn(y);  // 2p - y, limbs < 2^30: only S2's product reads it
    // the point is in registers before the next one overwrites its LDS quarters
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (j + 1 < kChunk) {
      if ((j + 1) % kDmaGroup == 0) stage((j + 1) / kDmaGroup);
      ent = sidx[((j + 1) % kDmaGroup) * kLdsStride + threadIdx.x];
      dma(ent);
    }
    if (pos < e) {
      if (use) acc_madd29(acc, inf, x, y, bases + (ent_cur & 0x7fffffffu), (ent_cur >> 31) != 0);
      const uint32_t p1 = pos + 1;
      if (p1 == kend || p1 == e) {
        const bool starts = kstart >= s;
        const bool ends = kend <= e;
        Xyzz29 out = acc;
        if (inf)
#pragma unroll
          for (int i = 0; i < 9; i++) out.ZZ.v[i] = 0;
        if (starts && ends) buckets[k] = out;
        else if (!starts) carry_cont[t] = out;
        else carry_own[t] = out;
        inf = true;
        while (p1 < e && kend <= p1) {
          k++;
          kstart = kend;
          kend = offsets[k + 1];
        }
      }
    }
  }
}

// ---- Batch-affine pairing rounds (fixed-base schedule) ---------------------------
// Before the XYZZ accumulation, R rounds halve every bucket's run in place of the
// sequential mixed additions: entries 2j and 2j+1 of a bucket's run become one affine
// point. An affine addition needs 1/(x2 - x1); the workgroup shares ONE Fermat
// inversion among all its pairs (Montgomery's trick: a prefix product per thread, a
// product tree over the workgroup's threads in LDS, then the prefixes unwound), so a
// pair costs 5 products + 1 square (3 for the trick, lambda, lambda^2, y3) against the
// 8 products + 2 squares of the XYZZ mixed addition (madd-2008-s), plus the tree and
// inversion shared by kPairThreads * kPairPer pairs. The exclusive prefixes go to a
// scratch array laid out [slot][limb][thread] (coalesced). Round 1 gathers the signed
// table entries through `sorted`; later rounds read the previous round's output.
// Pair slot p of bucket k (noff[k] <= p < noff[k+1], noff = exclusive scan of
// ceil(run/2), msm_pair_offsets_kernel) adds source positions off[k] + 2(p - noff[k])
// and the one after it, or copies the last entry of an odd run. Coordinates stay
// canonical Montgomery-261 (so the table's x == x' test finds doublings and P + (-P));
// infinity is (0, 0) as in the table.
// Opt-in (NZCB_PAIR_ROUNDS, nzcb_msm_set_pair_rounds): measured slower than the XYZZ
// accumulation alone at 2^21 (tried and dropped), kept parity-tested.

enum : uint32_t { kPairAdd = 0, kPairDbl = 1, kPairCopyA = 2, kPairCopyB = 3, kPairInf = 4 };

template <bool kGather>
__device__ __forceinline__ G1Affine pair_point(const G1Affine* __restrict__ src, const uint32_t* __restrict__ sorted,
                                               uint32_t pos) {
  if (!kGather) return src[pos];
  const uint32_t ent = sorted[pos];
  G1Affine P = src[ent & 0x7fffffffu];
  if ((ent >> 31) && !P.is_inf()) P.y = neg(P.y);
  return P;
}

__device__ __forceinline__ uint32_t pair_kind(const G1Affine& a, const G1Affine& b) {
  if (a.is_inf()) return kPairCopyB;
  if (b.is_inf()) return kPairCopyA;
  if (a.x == b.x) return a.y == b.y ? kPairDbl : kPairInf;
  return kPairAdd;
}

// denominator of the slope: x2 - x1, or 2 y1 for a doubling (y1 != 0 on BN254 G1)
__device__ __forceinline__ F29 pair_den(const G1Affine& a, const G1Affine& b, uint32_t kind) {
  return split29(kind == kPairAdd ? b.x - a.x : a.y + a.y);
}

// numerator of a doubling's slope, 3 x^2 (rare: kept out of line)
__device__ __noinline__ F29 pair_dbl_num(const Fq x) {
  const Fq xx = reduce_once(join29(sqr29(split29(x))));
  return split29(xx + xx + xx);
}

__device__ __forceinline__ uint32_t pm2_limb(int i) {  // limb i (radix 2^29) of p - 2
  switch (i) {
    case 0: return Fq29::P[0] - 2u;
    case 1: return Fq29::P[1];
    case 2: return Fq29::P[2];
    case 3: return Fq29::P[3];
    case 4: return Fq29::P[4];
    case 5: return Fq29::P[5];
    case 6: return Fq29::P[6];
    case 7: return Fq29::P[7];
    default: return Fq29::P[8];
  }
}

// a^(p-2) = a^-1 (Montgomery-261 in and out; a != 0 mod p), left-to-right binary powering
__device__ __noinline__ F29 inv29(const F29 a) {
  F29 r = f29_const(Fq29::ONE);
  for (int i = 8; i >= 0; i--) {
    const uint32_t e = pm2_limb(i);
    for (int b = (i == 8 ? 21 : 28); b >= 0; b--) {
      r = sqr29(r);
      if ((e >> b) & 1u) r = mul29(r, a);
    }
  }
  return r;
}

// noff[k] = sum_{j<k} ceil((off[j+1] - off[j]) / 2), noff[nkeys] = total (one workgroup)
__global__ void __launch_bounds__(1024)
msm_pair_offsets_kernel(const uint32_t* __restrict__ off, uint32_t nkeys, uint32_t* __restrict__ noff) {
  __shared__ uint32_t sh[1024];
  const uint32_t tid = threadIdx.x;
  const uint32_t per = (nkeys + 1023u) / 1024u;
  const uint32_t k0 = tid * per < nkeys ? tid * per : nkeys;
  const uint32_t k1 = k0 + per < nkeys ? k0 + per : nkeys;
  uint32_t sum = 0;
  for (uint32_t k = k0; k < k1; k++) sum += (off[k + 1] - off[k] + 1u) >> 1;
  sh[tid] = sum;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    const uint32_t v = tid >= d ? sh[tid - d] : 0u;
    __syncthreads();
    sh[tid] += v;
    __syncthreads();
  }
  uint32_t base = sh[tid] - sum;
  for (uint32_t k = k0; k < k1; k++) {
    noff[k] = base;
    base += (off[k + 1] - off[k] + 1u) >> 1;
  }
  if (tid == 1023) noff[nkeys] = sh[1023];
}

template <bool kGather>
__global__ void __launch_bounds__(kPairThreads)
msm_pair29_kernel(const G1Affine* __restrict__ src, const uint32_t* __restrict__ sorted,
                  const uint32_t* __restrict__ off, const uint32_t* __restrict__ noff, uint32_t nkeys,
                  uint32_t* __restrict__ pre, G1Affine* __restrict__ dst) {
  __shared__ F29 tree[2 * kPairThreads];
  const uint32_t total = noff[nkeys];
  if ((size_t)blockIdx.x * kPairThreads * kPairPer >= total) return;  // whole workgroup idle
  const uint32_t tid = threadIdx.x;
  const size_t nthr = (size_t)gridDim.x * kPairThreads;
  const size_t t = (size_t)blockIdx.x * kPairThreads + tid;
  const uint32_t p0 = (uint32_t)(t * kPairPer);
  const uint32_t p1 = p0 >= total ? p0 : (p0 + kPairPer < total ? p0 + kPairPer : total);
  uint32_t k = 0, ds = 0, de = 0, ss = 0, se = 0;  // bucket k: slots [ds, de), sources [ss, se)
  if (p0 < p1) {
    k = find_key(noff, nkeys, p0);
    ds = noff[k];
    de = noff[k + 1];
    ss = off[k];
    se = off[k + 1];
  }
  // forward: exclusive prefix products of the denominators
  F29 c = f29_const(Fq29::ONE);
  for (uint32_t p = p0; p < p1; p++) {
    while (p >= de) {
      k++;
      ds = de;
      de = noff[k + 1];
      ss = se;
      se = off[k + 1];
    }
    const uint32_t s = ss + 2u * (p - ds);
    if (s + 1u < se) {
      const G1Affine a = pair_point<kGather>(src, sorted, s), b = pair_point<kGather>(src, sorted, s + 1u);
      const uint32_t kind = pair_kind(a, b);
      if (kind <= kPairDbl) {
        uint32_t* q = pre + (size_t)(p - p0) * 9u * nthr + t;
#pragma unroll
        for (int l = 0; l < 9; l++) q[(size_t)l * nthr] = c.v[l];
        c = mul29(c, pair_den(a, b, kind));
      }
    }
  }
  // one inversion for the workgroup: product tree over the threads' totals
  tree[kPairThreads + tid] = c;
  __syncthreads();
  for (uint32_t w = kPairThreads / 2; w >= 1; w >>= 1) {
    if (tid < w) tree[w + tid] = mul29(tree[2 * (w + tid)], tree[2 * (w + tid) + 1]);
    __syncthreads();
  }
  if (tid == 0) tree[1] = inv29(tree[1]);
  __syncthreads();
  for (uint32_t w = 1; w < kPairThreads; w <<= 1) {
    if (tid < w) {
      const uint32_t nd = w + tid;
      const F29 iv = tree[nd], l = tree[2 * nd], r = tree[2 * nd + 1];
      tree[2 * nd] = mul29(iv, r);
      tree[2 * nd + 1] = mul29(iv, l);
    }
    __syncthreads();
  }
  F29 ic = tree[kPairThreads + tid];  // 1 / (product of this thread's denominators)
  // backward: unwind the prefixes, add the pairs
  for (uint32_t p = p1; p-- > p0;) {
    while (p < ds) {
      k--;
      de = ds;
      ds = noff[k];
      se = ss;
      ss = off[k];
    }
    const uint32_t s = ss + 2u * (p - ds);
    const G1Affine a = pair_point<kGather>(src, sorted, s);
    G1Affine out = a;
    if (s + 1u < se) {
      const G1Affine b = pair_point<kGather>(src, sorted, s + 1u);
      const uint32_t kind = pair_kind(a, b);
      if (kind <= kPairDbl) {
        const uint32_t* q = pre + (size_t)(p - p0) * 9u * nthr + t;
        F29 e;
#pragma unroll
        for (int l = 0; l < 9; l++) e.v[l] = q[(size_t)l * nthr];
        const F29 id = mul29(ic, e);  // 1 / den
        ic = mul29(ic, pair_den(a, b, kind));
        const F29 num = kind == kPairAdd ? split29(b.y - a.y) : pair_dbl_num(a.x);
        const F29 lam = mul29(num, id);
        const Fq x2 = kind == kPairAdd ? b.x : a.x;
        out.x = reduce_once(join29(sqr29(lam))) - a.x - x2;
        out.y = reduce_once(join29(mul29(lam, split29(a.x - out.x)))) - a.y;
      } else if (kind == kPairCopyB) {
        out = b;
      } else if (kind == kPairInf) {
        out.x = Fq::zero();
        out.y = Fq::zero();
      }
    }
    dst[p] = out;
  }
}

// Kernels below keep exactly one inlined EC addition per loop body: an inlined
// formula is ~3.5k instructions, and several copies in one loop thrash the shared
// instruction cache (measured: 2.7 ms -> see profiles/ for the single-site form).

// Buckets whose entries span several accumulation chunks: owner chunk's carry plus
// the continuation carries of the chunks the bucket spills into (thread per bucket).
// sum of a bucket's carries: the owner chunk's and the continuations c0+1..c1
__device__ __forceinline__ G1xyzz sum_run(const G1xyzz* carry_own, const G1xyzz* carry_cont, uint32_t c0,
                                          uint32_t c1) {
  G1xyzz v = carry_own[c0];
  for (uint32_t u = c0 + 1; u <= c1; u++) v = xyzz_add(v, carry_cont[u]);
  return v;
}
// radix-2^29 carries are summed in that radix (no per-carry conversion), converted once
__device__ __forceinline__ G1xyzz sum_run(const Xyzz29* carry_own, const Xyzz29* carry_cont, uint32_t c0,
                                          uint32_t c1) {
  Xyzz29 v = carry_own[c0];
  for (uint32_t u = c0 + 1; u <= c1; u++) v = add29(v, carry_cont[u]);
  return load_point(v);
}

// P = G1xyzz: the generic accumulation already wrote single-chunk buckets in place;
// P = Xyzz29: with out29 the multi-chunk buckets are summed into out29 (= the
// accumulation's bucket array, single-chunk buckets stay where it wrote them, nothing is
// converted: msm_bitsums29_kernel reads radix 2^29); without, every bucket is converted
// into `buckets` (single-chunk ones from `single`).
template <class P>
__global__ void __launch_bounds__(kMsmThreads)
msm_bucket_finalize_kernel(uint32_t chunk, const uint32_t* __restrict__ offsets, uint32_t nkeys, uint32_t seq_span29,
                           const P* __restrict__ single,
                           const P* __restrict__ carry_own, const P* __restrict__ carry_cont,
                           G1xyzz* __restrict__ buckets, uint32_t* __restrict__ large, Xyzz29* __restrict__ out29) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nkeys) return;
  const uint32_t s = offsets[k], e = offsets[k + 1];
  if (e == s) return;
  const uint32_t c0 = s / chunk, c1 = (e - 1) / chunk;
  if (c0 == c1) {  // stored by the accumulation
    if (single && !out29) buckets[k] = load_point(single[k]);
    return;
  }
  if (c1 - c0 > (std::is_same<P, Xyzz29>::value ? seq_span29 : kSeqSpan)) {  // long run (skewed digits)
    large[1 + atomicAdd(&large[0], 1u)] = (uint32_t)k;
    return;
  }
  if constexpr (std::is_same<P, Xyzz29>::value) {
    if (out29) {
      Xyzz29 v = carry_own[c0];
      for (uint32_t u = c0 + 1; u <= c1; u++) v = add29(v, carry_cont[u]);
      out29[k] = v;
      return;
    }
  }
  buckets[k] = sum_run(carry_own, carry_cont, c0, c1);
}

// thread per (set, L-bucket segment): run = sum_j B_j, tot = sum_j (j+1) B_j
__global__ void __launch_bounds__(kMsmThreads)
msm_bucket_reduce_kernel(const G1xyzz* __restrict__ buckets, const uint32_t* __restrict__ offsets, int nb,
                         int seglen, int nseg, int nsets, G1xyzz* __restrict__ seg_tot, G1xyzz* __restrict__ seg_run) {
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)nsets * nseg) return;
  const int w = (int)(t / nseg);
  const int g = (int)(t % nseg);
  const size_t base = (size_t)w * nb + (size_t)g * seglen;
  G1xyzz run = G1xyzz::inf(), tot = G1xyzz::inf();
  for (int j = seglen - 1; j >= 0; j--) {  // two addition sites, no selected operand (scratch)
    const uint32_t k = (uint32_t)(base + j);
    if (offsets[k + 1] != offsets[k]) run = xyzz_add(run, buckets[k]);
    if (!run.is_inf()) tot = xyzz_add(tot, run);
  }
  seg_tot[t] = tot;  // sum_j (j+1) * bucket_{g*L+j}
  seg_run[t] = run;  // sum_j bucket_{g*L+j}
}

// point addition / infinity for the block sums: 8x32 XYZZ (G1xyzz) or radix-2^29 (Xyzz29)
__device__ __forceinline__ G1xyzz padd(const G1xyzz& a, const G1xyzz& b) { return xyzz_add(a, b); }
__device__ __forceinline__ Xyzz29 padd(const Xyzz29& a, const Xyzz29& b) { return add29(a, b); }
template <class P> __device__ __forceinline__ P pinf();
template <> __device__ __forceinline__ G1xyzz pinf<G1xyzz>() { return G1xyzz::inf(); }
template <> __device__ __forceinline__ Xyzz29 pinf<Xyzz29>() {
  Xyzz29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.X.v[i] = r.Y.v[i] = r.ZZ.v[i] = r.ZZZ.v[i] = 0;
  return r;
}

// Block tree sum with a single EC-addition site: `per` sequential steps in which
// load(step, rhs) supplies the thread's next term, then log2(T) LDS tree levels.
template <int T, class Load, class Pt = G1xyzz>
__device__ __forceinline__ Pt block_sum(int per, Pt* sh, Load&& load) {
  constexpr int LG = T == 256 ? 8 : T == 128 ? 7 : T == 64 ? 6 : 5;
  const int tid = threadIdx.x;
  Pt acc = pinf<Pt>();
  for (int step = 0; step < per + LG; step++) {
    if (step == per) {
      sh[tid] = acc;
      __syncthreads();
    }
    bool doit;
    Pt lhs, rhs;
    if (step < per) {
      doit = load(step, rhs);
      lhs = acc;
    } else {
      const int stride = (T >> 1) >> (step - per);
      doit = tid < stride;
      if (doit) {
        lhs = sh[tid];
        rhs = sh[tid + stride];
      }
    }
    Pt r;
    if (doit) r = padd(lhs, rhs);
    if (step < per) {
      if (doit) acc = r;
    } else {
      if (doit) sh[tid] = r;
      __syncthreads();
    }
  }
  return sh[0];
}

// Fixed base with radix-2^29 sums (out29), opt-in (NZCB_FIN_LANES=4): four lanes per
// bucket, lane r adds the carries c0 + r, c0 + r + 4, ..., then two xor-shuffle levels join
// the lanes: ~span / 4 + 2 dependent additions instead of span - 1 (isolated finalize
// 0.185 -> 0.152 ms at 2^21), but every lane of a wave issues each addition: 55.9 M VALU
// instructions per launch against 36.5 M sequential (profiles/r3_fin_valu.txt), and the
// 5-lane bench is VALU-bound, so the sequential sum stays the default. Single-chunk
// buckets are already in place; runs longer than kSeqSpan29 carries go to the large list.
__device__ __forceinline__ Xyzz29 shfl_xor29(const Xyzz29& v, int m) {
  Xyzz29 o;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    o.X.v[i] = __shfl_xor(v.X.v[i], m);
    o.Y.v[i] = __shfl_xor(v.Y.v[i], m);
    o.ZZ.v[i] = __shfl_xor(v.ZZ.v[i], m);
    o.ZZZ.v[i] = __shfl_xor(v.ZZZ.v[i], m);
  }
  return o;
}

__global__ void __launch_bounds__(kMsmThreads)
msm_finalize29_kernel(uint32_t chunk, const uint32_t* __restrict__ offsets, uint32_t nkeys,
                      const Xyzz29* __restrict__ carry_own, const Xyzz29* __restrict__ carry_cont,
                      uint32_t* __restrict__ large, Xyzz29* __restrict__ out29) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t k = t >> 2;
  const uint32_t r = (uint32_t)t & 3u;
  bool multi = false;  // the same for the bucket's four lanes
  uint32_t c0 = 0, c1 = 0;
  if (k < nkeys) {
    const uint32_t s = offsets[k], e = offsets[k + 1];
    if (e != s) {
      c0 = s / chunk;
      c1 = (e - 1) / chunk;
      if (c1 - c0 > kSeqSpan29) {
        if (r == 0) large[1 + atomicAdd(&large[0], 1u)] = (uint32_t)k;
      } else {
        multi = c1 > c0;
      }
    }
  }
  Xyzz29 v = pinf<Xyzz29>();
  if (multi)
    for (uint32_t u = c0 + r; u <= c1; u += 4) v = add29(v, u == c0 ? carry_own[c0] : carry_cont[u]);
#pragma unroll 1
  for (int m = 1; m <= 2; m <<= 1) {  // every lane shuffles (no divergence around the exchange)
    const Xyzz29 o = shfl_xor29(v, m);
    if (multi) v = add29(v, o);
  }
  if (multi && r == 0) out29[k] = v;
}

// Buckets listed by the finalize kernel (more than kSeqSpan carries, e.g. many equal
// digits): one workgroup per bucket, kSumThreads-way partial sums + LDS tree.
template <class P>
__global__ void __launch_bounds__(kSumThreads)
msm_bucket_large_kernel(uint32_t chunk, const uint32_t* __restrict__ offsets, const uint32_t* __restrict__ large,
                        const P* __restrict__ carry_own, const P* __restrict__ carry_cont,
                        G1xyzz* __restrict__ buckets) {
  __shared__ G1xyzz sh[kSumThreads];
  const uint32_t count = large[0];
  for (uint32_t i = blockIdx.x; i < count; i += gridDim.x) {
    const uint32_t k = large[1 + i];
    const uint32_t c0 = offsets[k] / chunk, c1 = (offsets[k + 1] - 1) / chunk;
    const uint32_t span = c1 - c0 + 1;
    const int per = (int)((span + kSumThreads - 1) / kSumThreads);
    const G1xyzz r = block_sum<kSumThreads>(per, sh, [&](int step, G1xyzz& rhs) {
      const uint32_t u = (uint32_t)step * kSumThreads + threadIdx.x;
      if (u >= span) return false;
      rhs = load_point(u ? carry_cont[c0 + u] : carry_own[c0]);
      return true;
    });
    if (threadIdx.x == 0) buckets[k] = r;
    __syncthreads();
  }
}

// Fixed-base schedule, long carry runs (e.g. the Lagrange-basis commitments, whose small
// witness values put ~40 % of the entries in bucket 0: ~12 k carries): the runs are cut
// into pieces of kPieceCarries, each summed by one workgroup in radix 2^29 (kSumPer-deep
// sequential adds + LDS tree), then one thread per bucket adds its pieces. One workgroup
// per bucket (msm_bucket_large_kernel) took ~40 dependent additions plus conversions.
static constexpr uint32_t kPieceCarries = (uint32_t)kSumThreads * kSumPer;

__device__ __forceinline__ uint32_t carry_span(uint32_t chunk, const uint32_t* offsets, uint32_t k, uint32_t* c0) {
  *c0 = offsets[k] / chunk;
  return (offsets[k + 1] - 1) / chunk - *c0 + 1;
}

// off[i] = pieces of the listed buckets before i, off[count] = all (one workgroup)
__global__ void __launch_bounds__(1024)
msm_large_scan_kernel(uint32_t chunk, const uint32_t* __restrict__ offsets, const uint32_t* __restrict__ large,
                      uint32_t* __restrict__ off) {
  __shared__ uint32_t sh[1024];
  const uint32_t count = large[0];
  const uint32_t tid = threadIdx.x;
  const uint32_t per = (count + 1023u) / 1024u;
  const uint32_t i0 = tid * per < count ? tid * per : count;
  const uint32_t i1 = i0 + per < count ? i0 + per : count;
  auto pieces = [&](uint32_t i) {
    uint32_t c0;
    return (carry_span(chunk, offsets, large[1 + i], &c0) + kPieceCarries - 1) / kPieceCarries;
  };
  uint32_t sum = 0;
  for (uint32_t i = i0; i < i1; i++) sum += pieces(i);
  sh[tid] = sum;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    const uint32_t v = tid >= d ? sh[tid - d] : 0u;
    __syncthreads();
    sh[tid] += v;
    __syncthreads();
  }
  uint32_t base = sh[tid] - sum;
  for (uint32_t i = i0; i < i1; i++) {
    off[i] = base;
    base += pieces(i);
  }
  if (tid == 1023) off[count] = sh[1023];
}

__global__ void __launch_bounds__(kSumThreads)
msm_large_piece29_kernel(uint32_t chunk, const uint32_t* __restrict__ offsets, const uint32_t* __restrict__ large,
                         const uint32_t* __restrict__ off, const Xyzz29* __restrict__ carry_own,
                         const Xyzz29* __restrict__ carry_cont, Xyzz29* __restrict__ part) {
  __shared__ Xyzz29 sh[kSumThreads];
  const uint32_t count = large[0];
  const uint32_t total = off[count];
  for (uint32_t item = blockIdx.x; item < total; item += gridDim.x) {
    uint32_t lo = 0, hi = count;  // largest i with off[i] <= item
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (off[mid] <= item) lo = mid; else hi = mid;
    }
    uint32_t c0;
    const uint32_t span = carry_span(chunk, offsets, large[1 + lo], &c0);
    const uint32_t first = (item - off[lo]) * kPieceCarries;
    const uint32_t n = span - first < kPieceCarries ? span - first : kPieceCarries;
    const int per = (int)((n + kSumThreads - 1) / kSumThreads);  // <= kSumPer
    const Xyzz29 r = block_sum<kSumThreads>(per, sh, [&](int step, Xyzz29& rhs) {
      const uint32_t u = (uint32_t)step * kSumThreads + threadIdx.x;
      if (u >= n) return false;
      rhs = first + u ? carry_cont[c0 + first + u] : carry_own[c0];
      return true;
    });
    if (threadIdx.x == 0) part[item] = r;
    __syncthreads();
  }
}

// a listed bucket's pieces: one wave per bucket, a tree over up to 64 pieces at a time
// (the hottest Lagrange bucket has ~40 pieces: 6 levels instead of 40 sequential adds)
__global__ void __launch_bounds__(kLargeFinalThreads)
msm_large_final29_kernel(const uint32_t* __restrict__ large, const uint32_t* __restrict__ off,
                         const Xyzz29* __restrict__ part, G1xyzz* __restrict__ buckets, Xyzz29* __restrict__ out29) {
  __shared__ Xyzz29 sh[kLargeFinalThreads];
  const uint32_t count = large[0];
  for (uint32_t i = blockIdx.x; i < count; i += gridDim.x) {
    const uint32_t p0 = off[i], np = off[i + 1] - p0;
    if (np == 1) {
      if (threadIdx.x == 0) {
        if (out29) out29[large[1 + i]] = part[p0];
        else buckets[large[1 + i]] = load_point(part[p0]);
      }
      continue;
    }
    const int per = (int)((np + kLargeFinalThreads - 1) / kLargeFinalThreads);
    const Xyzz29 r = block_sum<kLargeFinalThreads>(per, sh, [&](int step, Xyzz29& rhs) {
      const uint32_t u = (uint32_t)step * kLargeFinalThreads + threadIdx.x;
      if (u >= np) return false;
      rhs = part[p0 + u];
      return true;
    });
    if (threadIdx.x == 0) {
      if (out29) out29[large[1 + i]] = r;
      else buckets[large[1 + i]] = load_point(r);
    }
    __syncthreads();
  }
}

// level 1: block (set w, slot j, part p). Slot 0 sums seg_tot[w][g] over all g; slot b+1
// sums seg_run[w][g] over the g with bit b set. Part p covers kSumPer * T terms.
__global__ void __launch_bounds__(kSumThreads)
msm_sums_kernel(const G1xyzz* __restrict__ seg_tot, const G1xyzz* __restrict__ seg_run, int nseg, int nslots,
                int nparts, G1xyzz* __restrict__ parts) {
  __shared__ G1xyzz sh[kSumThreads];
  const int p = blockIdx.x % nparts;
  const int wj = blockIdx.x / nparts;
  const int j = wj % nslots;
  const int w = wj / nslots;
  const int count = j == 0 ? nseg : nseg >> 1;
  const G1xyzz r = block_sum<kSumThreads>(kSumPer, sh, [&](int step, G1xyzz& rhs) {
    const int q = (p * kSumPer + step) * kSumThreads + (int)threadIdx.x;
    if (q >= count) return false;
    int g = q;
    if (j) {
      const int b = j - 1;
      g = ((q >> b) << (b + 1)) | (1 << b) | (q & ((1 << b) - 1));
    }
    rhs = j ? seg_run[(size_t)w * nseg + g] : seg_tot[(size_t)w * nseg + g];
    return true;
  });
  if (threadIdx.x == 0) parts[blockIdx.x] = r;
}

// level 2: block per (set, slot) sums its nparts partials
__global__ void __launch_bounds__(kPartThreads)
msm_parts_kernel(const G1xyzz* __restrict__ parts, int nparts, G1xyzz* __restrict__ out) {
  __shared__ G1xyzz sh[kPartThreads];
  const int per = (nparts + kPartThreads - 1) / kPartThreads;
  const G1xyzz r = block_sum<kPartThreads>(per, sh, [&](int step, G1xyzz& rhs) {
    const int q = step * kPartThreads + (int)threadIdx.x;
    if (q >= nparts) return false;
    rhs = parts[(size_t)blockIdx.x * nparts + q];
    return true;
  });
  if (threadIdx.x == 0) out[blockIdx.x] = r;
}

// Fixed base (one bucket set of nb = 2^lb buckets, bucket k of weight k + 1): the window
// sum sum_k (k + 1) B_k = sum_b 2^b S_b with S_b = sum of the buckets whose weight has
// bit b set (b = 0..lb; slot lb holds bucket nb - 1 alone). Block (slot b, part p) sums
// kSumPer * kSumThreads of slot b's terms: 4 sequential additions + an 8-level tree, in
// radix 2^29 on the accumulation's own bucket array. The segment reduce of the generic
// schedule (msm_bucket_reduce_kernel: 16 dependent 8x32 additions per thread, 2^13
// threads, then msm_sums_kernel) did 1/4 of the additions in a 3x longer dependency
// chain; both are latency-bound at this size (profiles/r3_single_lane_phases.txt).
__global__ void __launch_bounds__(kSumThreads)
msm_bitsums29_kernel(const Xyzz29* __restrict__ buckets, const uint32_t* __restrict__ offsets, int lb, int nparts,
                     Xyzz29* __restrict__ parts) {
  __shared__ Xyzz29 sh[kSumThreads];
  const int p = blockIdx.x % nparts;
  const int b = blockIdx.x / nparts;
  const uint32_t count = b < lb ? 1u << (lb - 1) : 1u;
  const Xyzz29 r = block_sum<kSumThreads>(kSumPer, sh, [&](int step, Xyzz29& rhs) {
    const uint32_t q = (uint32_t)(p * kSumPer + step) * kSumThreads + threadIdx.x;
    if (q >= count) return false;
    const uint32_t v = b < lb ? (((q >> b) << (b + 1)) | (1u << b) | (q & ((1u << b) - 1u))) : 1u << lb;
    const uint32_t k = v - 1u;  // weight v
    if (offsets[k + 1] == offsets[k]) return false;
    rhs = buckets[k];
    return true;
  });
  if (threadIdx.x == 0) parts[blockIdx.x] = r;
}

// Default fixed-base sums, two levels in radix 2^29. Level 1, thread per segment g of
// kSeg29 buckets: run_g = sum_j B_{g L + j}, tot_g = sum_j (j + 1) B_{g L + j} (running
// sums from the top: 2 L dependent additions). Level 2 (msm_segsums29_kernel): slot 0 =
// sum_g tot_g, slot 1 + b = sum of run_g over the g with bit b set, so that the window sum
// is slot 0 + L sum_b 2^b slot_{1+b} (msm_finish). Each bucket is added twice and each
// segment ~log2(nseg) / 2 + 1 times: ~2.0 additions per bucket against ~8 for the bit slots
// over the buckets, with a dependency chain of 2 L + 4 + 8 (+ 7 in msm_parts29_kernel).
static constexpr int kSeg29 = 4;

__global__ void __launch_bounds__(kMsmThreads)
msm_seg29_kernel(const Xyzz29* __restrict__ buckets, const uint32_t* __restrict__ offsets, uint32_t nseg,
                 Xyzz29* __restrict__ seg_tot, Xyzz29* __restrict__ seg_run) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nseg) return;
  Xyzz29 run = pinf<Xyzz29>(), tot = pinf<Xyzz29>();
  for (int j = kSeg29 - 1; j >= 0; j--) {  // two addition sites per step
    const uint32_t k = g * kSeg29 + (uint32_t)j;
    if (offsets[k + 1] != offsets[k]) run = add29(run, buckets[k]);
    tot = add29(tot, run);
  }
  seg_tot[g] = tot;
  seg_run[g] = run;
}

// block (slot j, part p): slot 0 sums seg_tot[0..nseg), slot b + 1 the seg_run[g] with
// bit b of g set; part p covers kSumPer * kSumThreads terms
__global__ void __launch_bounds__(kSumThreads)
msm_segsums29_kernel(const Xyzz29* __restrict__ seg_tot, const Xyzz29* __restrict__ seg_run, int nseg, int nparts,
                     Xyzz29* __restrict__ parts) {
  __shared__ Xyzz29 sh[kSumThreads];
  const int p = blockIdx.x % nparts;
  const int j = blockIdx.x / nparts;
  const int count = j == 0 ? nseg : nseg >> 1;
  const Xyzz29 r = block_sum<kSumThreads>(kSumPer, sh, [&](int step, Xyzz29& rhs) {
    const int q = (p * kSumPer + step) * kSumThreads + (int)threadIdx.x;
    if (q >= count) return false;
    if (j == 0) {
      rhs = seg_tot[q];
    } else {
      const int b = j - 1;
      rhs = seg_run[((q >> b) << (b + 1)) | (1 << b) | (q & ((1 << b) - 1))];
    }
    return true;
  });
  if (threadIdx.x == 0) parts[blockIdx.x] = r;
}

// block per slot: its nparts partials, converted to the 8x32 layout once
__global__ void __launch_bounds__(kPartThreads)
msm_parts29_kernel(const Xyzz29* __restrict__ parts, int nparts, G1xyzz* __restrict__ out) {
  __shared__ Xyzz29 sh[kPartThreads];
  const int per = (nparts + kPartThreads - 1) / kPartThreads;
  const Xyzz29 r = block_sum<kPartThreads>(per, sh, [&](int step, Xyzz29& rhs) {
    const int q = step * kPartThreads + (int)threadIdx.x;
    if (q >= nparts) return false;
    rhs = parts[(size_t)blockIdx.x * nparts + q];
    return true;
  });
  if (threadIdx.x == 0) out[blockIdx.x] = load_point(r);
}

// Shifted-base table: row w = 2^(c*w) * B_i, thread per base (c doublings per row,
// one Fermat inversion per stored affine point). fold: the rows of 2^-256 B_i instead
// (kinv = 2^-256 mod r as an integer), so that the Montgomery-256 form m = s 2^256 of a
// scalar is itself the digit source: sum m_i (2^-256 B_i) = sum s_i B_i, and the MSM's
// two digit passes skip their from_mont_fr29 product per scalar.
__global__ void __launch_bounds__(kMsmThreads)
msm_table_kernel(const G1Affine* __restrict__ bases, size_t n, size_t stride, int c, int nw, Fq k261, int fold,
                 Fr kinv, G1Affine* __restrict__ q) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const G1Affine P = bases[i];
  if (P.is_inf()) {
    for (int w = 0; w < nw; w++) q[(size_t)w * stride + i] = P;
    return;
  }
  G1xyzz acc = xyzz_from_affine(P);
  if (fold) {  // 2^-256 P, left-to-right double-and-add (kinv < r < 2^254, uniform bits)
    acc = G1xyzz::inf();
    for (int b = 253; b >= 0; b--) {
      acc = xyzz_dbl(acc);
      if ((kinv.v[b >> 5] >> (b & 31)) & 1u) acc = xyzz_add_affine(acc, P.x, P.y);
    }
  }
  for (int w = 0; w < nw; w++) {
    if (w)
      for (int k = 0; k < c; k++) acc = xyzz_dbl(acc);
    const Fq ti = inverse(acc.ZZ * acc.ZZZ);
    G1Affine r;  // affine, Montgomery-261 (x * 2^261 = mont256(x * 2^256, 2^261))
    r.x = acc.X * (acc.ZZZ * ti) * k261;
    r.y = acc.Y * (acc.ZZ * ti) * k261;
    q[(size_t)w * stride + i] = r;
  }
}

void MsmBaseTable::build(const G1Affine* bases, size_t npts, int cbits, hipStream_t st, bool fold_mont) {
  n = npts;
  mont_folded = fold_mont;
  stride = npts;
  c = cbits;
  nw = num_windows(c);
  if ((size_t)nw * stride >= (size_t(1) << 31)) throw Error(NZCB_ERR_ARG, "msm table too large for 31-bit indices");
  q.alloc((size_t)nw * stride + 1);  // + the infinity point zero digits point at
  NZ_HIP(hipMemsetAsync(q.p + (size_t)nw * stride, 0, sizeof(G1Affine), st));
  Fq thirty_two = Fq::zero();
  thirty_two.v[0] = 32;
  const Fq k261 = to_mont(thirty_two);  // 2^261 mod p
  Fr one_raw = Fr::zero();
  one_raw.v[0] = 1;
  const Fr kinv = from_mont(one_raw);  // the integer 2^-256 mod r
  hipLaunchKernelGGL(msm_table_kernel, dim3(grid_for(n, kMsmThreads, 1u << 30)), dim3(kMsmThreads), 0, st, bases, n,
                     stride, c, nw, k261, fold_mont ? 1 : 0, kinv, q.p);
  NZ_HIP(hipGetLastError());
}

// work items of the bucket_lo steps: at most one partial segment per region + entries / kLoSeg
static size_t lo_items_bound(size_t entries) { return 256 + entries / kLoSeg + 1; }

struct MsmPlan {
  int c, nw, nsets, seglen, nseg, nbits, nslots, nparts;
  int lb, bparts;  // fixed base, bit-slot sums: log2(nb) (slots lb + 1), parts per slot
  int nseg29, nslots29, sparts29;  // fixed base, segment sums: segments, slots, parts per slot
  uint32_t nb, nkeys;
  size_t entries;
};

static MsmPlan make_plan(size_t n, const MsmBaseTable* t) {
  MsmPlan p;
  p.c = t ? t->c : msm_window_bits(n);
  p.nw = num_windows(p.c);
  p.nsets = t ? 1 : p.nw;
  p.nb = 1u << (p.c - 1);
  p.nkeys = p.nb * (uint32_t)p.nsets;
  p.seglen = (int)(p.nb < (uint32_t)kSegLen ? p.nb : kSegLen);
  p.nseg = (int)(p.nb / p.seglen);
  p.nbits = 0;
  while ((1 << p.nbits) < p.nseg) p.nbits++;
  p.nslots = p.nbits + 1;
  p.nparts = (p.nseg + kSumThreads * kSumPer - 1) / (kSumThreads * kSumPer);
  p.lb = p.c - 1;
  p.bparts = (int)(((p.nb >> 1) + kSumThreads * kSumPer - 1) / (kSumThreads * kSumPer));
  p.nseg29 = (int)(p.nb >= (uint32_t)kSeg29 ? p.nb / kSeg29 : 1);
  p.nslots29 = 1;
  while ((1 << (p.nslots29 - 1)) < p.nseg29) p.nslots29++;
  p.sparts29 = (p.nseg29 + kSumThreads * kSumPer - 1) / (kSumThreads * kSumPer);
  p.entries = n * (size_t)p.nw;
  return p;
}

void MsmScratch::init(size_t maxp, bool fixed_base) {
  max_points = maxp;
  size_t max_entries = 0, max_keys = 0, max_seg = 0, max_slots = 0, max_parts = 0, max_parts29 = 0, max_seg29 = 0;
  auto fit = [&](const MsmPlan& p) {
    max_entries = std::max(max_entries, p.entries);
    max_keys = std::max(max_keys, (size_t)p.nkeys);
    max_seg = std::max(max_seg, (size_t)p.nseg * p.nsets);
    max_slots = std::max(max_slots, (size_t)p.nslots * p.nsets);
    max_parts = std::max(max_parts, (size_t)p.nslots * p.nsets * p.nparts);
    if (p.nsets == 1) {  // fixed base: the bit-slot sums
      max_slots = std::max(max_slots, (size_t)std::max(p.lb + 1, p.nslots29));
      max_parts29 = std::max(max_parts29, (size_t)std::max((p.lb + 1) * p.bparts, p.nslots29 * p.sparts29));
      max_seg29 = std::max(max_seg29, (size_t)p.nseg29);
    }
  };
  for (size_t n = 1;; n <<= 1) {
    size_t m = n < maxp ? n : maxp;
    fit(make_plan(m, nullptr));
    if (m == maxp) break;
  }
  if (fixed_base) {  // the PTau tables' window and the Lagrange table's
    MsmBaseTable t;
    t.c = fixed_base_window();
    fit(make_plan(maxp, &t));
    t.c = lagrange_window();
    fit(make_plan(maxp, &t));
  }
  offsets.alloc(max_keys + 1);
  sorted.alloc(max_entries);
  keys_in.alloc(max_entries);
  keys_out.alloc(max_entries);
  vals_in.alloc(max_entries);
  sort_tmp_bytes = 0;
  radix_sort(nullptr, sort_tmp_bytes, keys_in.p, keys_out.p, vals_in.p, sorted.p, max_entries, 21, nullptr);
  size_t tmp16 = 0;
  radix_sort(nullptr, tmp16, (const uint16_t*)keys_in.p, (uint16_t*)keys_out.p, vals_in.p, sorted.p, max_entries, 16,
             nullptr);
  sort_tmp_bytes = std::max(sort_tmp_bytes, tmp16);
  sort_tmp.alloc(sort_tmp_bytes + 16);
  buckets.alloc(max_keys);
  size_t nthreads = (max_entries + kMinChunk - 1) / kMinChunk + 1;  // the smallest chunk chunk_for allows
  carry_own.alloc(nthreads);
  large.alloc(max_keys + 1);
  if (fixed_base) {
    MsmBaseTable t;
    t.c = fixed_base_window();
    MsmPlan fp = make_plan(maxp, &t);
    t.c = lagrange_window();
    const MsmPlan lp = make_plan(maxp, &t);
    if (lp.entries > fp.entries) fp = lp;
    const size_t b1 = pair_bound(fp.entries, std::min(fp.nkeys, lp.nkeys)), b2 = pair_bound(b1, std::min(fp.nkeys, lp.nkeys));
    pair_pts[0].alloc(b1 ? b1 : 1);
    pair_pts[1].alloc(b2 ? b2 : 1);
    pair_off[0].alloc((size_t)max_keys + 1);
    pair_off[1].alloc((size_t)max_keys + 1);
    pair_pre.alloc(pair_grid(b1) * kPairThreads * kPairPer * 9);
    buckets29.alloc(max_keys);
    large_off.alloc(max_keys + 2);
    // pieces: sum over listed buckets of ceil(span / kPieceCarries) <= chunks / kPieceCarries + buckets
    large_part.alloc(nthreads / kPieceCarries + max_keys + 1);
    carry_own29.alloc(nthreads);
    carry_cont29.alloc(nthreads);
    parts29.alloc(max_parts29);
    seg_tot29.alloc(max_seg29);
    seg_run29.alloc(max_seg29);
    bin_counts.alloc((size_t)256 * ((maxp + kTileScalars - 1) / kTileScalars) + 256);  // + row totals
    vals_mid.alloc(max_entries);
    lo_seg.alloc(lo_items_bound(max_entries) * ((size_t)1 << BinKeys<20>::LO));  // the widest low index
  }
  carry_cont.alloc(nthreads);
  seg_tot.alloc(max_seg);
  seg_run.alloc(max_seg);
  parts.alloc(max_parts);
  win.alloc(max_slots);
  host_win_cap = max_slots;
  NZ_HIP(hipHostMalloc((void**)&host_win, max_slots * sizeof(G1xyzz), hipHostMallocDefault));
}

MsmScratch::~MsmScratch() {
  if (host_win) (void)hipHostFree(host_win);
  if (done) (void)hipEventDestroy(done);
  for (auto& e : ev)
    if (e) (void)hipEventDestroy(e);
}

template <int C, bool FIXED, class K = uint32_t>
static void launch_keys(const Fr* scalars, size_t n, int mont, size_t stride, MsmScratch& sc, hipStream_t st,
                        uint32_t skip_val = 0) {
  hipLaunchKernelGGL((msm_keys_kernel<C, FIXED, K>), dim3(grid_for(n, kMsmThreads, 1u << 30)), dim3(kMsmThreads), 0,
                     st, scalars, n, mont, stride, skip_val, (K*)sc.keys_in.p, sc.vals_in.p);
  NZ_HIP(hipGetLastError());
}

static void keys_dispatch(int c, const Fr* scalars, size_t n, int mont, const MsmBaseTable* t, MsmScratch& sc,
                          hipStream_t st) {
  if (t) {
    const uint32_t inf_idx = (uint32_t)((size_t)t->nw * t->stride);  // the table's infinity point
    switch (c) {
      case 16: launch_keys<16, true, uint16_t>(scalars, n, mont, t->stride, sc, st, inf_idx); return;
      case 17: launch_keys<17, true, uint16_t>(scalars, n, mont, t->stride, sc, st, inf_idx); return;
      case 18: launch_keys<18, true>(scalars, n, mont, t->stride, sc, st); return;
      case 19: launch_keys<19, true>(scalars, n, mont, t->stride, sc, st); return;
      case 20: launch_keys<20, true>(scalars, n, mont, t->stride, sc, st); return;
      default: throw Error(NZCB_ERR_INTERNAL, "bad fixed-base msm window");
    }
  }
  switch (c) {
#define NZ_CASE(K) case K: launch_keys<K, false>(scalars, n, mont, 0, sc, st); break;
    NZ_CASE(4) NZ_CASE(5) NZ_CASE(6) NZ_CASE(7) NZ_CASE(8) NZ_CASE(9) NZ_CASE(10) NZ_CASE(11) NZ_CASE(12)
    NZ_CASE(13) NZ_CASE(14) NZ_CASE(15) NZ_CASE(16)
#undef NZ_CASE
    default: throw Error(NZCB_ERR_INTERNAL, "bad msm window");
  }
}

G1Affine xyzz_to_affine(const G1xyzz& p) {
  G1Affine r;
  if (p.is_inf()) {
    r.x = Fq::zero();
    r.y = Fq::zero();
    return r;
  }
  r.x = p.X * inverse(p.ZZ);
  r.y = p.Y * inverse(p.ZZZ);
  return r;
}

void msm_enqueue(MsmScratch& sc, const G1Affine* bases, const Fr* scalars, size_t n, bool mont, hipStream_t st,
                 const MsmBaseTable* table) {
  sc.cur_n = n;
  if (n == 0) return;
  if (!sc.done) NZ_HIP(hipEventCreateWithFlags(&sc.done, hipEventDisableTiming));
  if (n > sc.max_points) throw Error(NZCB_ERR_ARG, "msm larger than scratch");
  if (table && n > table->n) throw Error(NZCB_ERR_ARG, "msm larger than its base table");
  if (table && table->mont_folded && !mont) throw Error(NZCB_ERR_ARG, "2^-256-folded table needs Montgomery scalars");
  // a folded table takes the Montgomery form's integer as the scalar (msm_table_kernel)
  const int mdig = (mont && !(table && table->mont_folded)) ? 1 : 0;
  const MsmPlan p = make_plan(n, table);
  if (p.entries > sc.sorted.n || p.nkeys + 1 > sc.offsets.n)
    throw Error(NZCB_ERR_ARG, "msm scratch was not sized for this schedule");
  const G1Affine* gather = table ? table->q.p : bases;
  sc.cur_c = p.c;
  sc.cur_nsets = p.nsets;
  sc.cur_nbits = p.nbits;
  sc.cur_seglen = p.seglen;
  sc.cur_nkeys = p.nkeys;
  const int fsums = table ? fb_sums() : 0;  // 0: the generic 8x32 sums
  const bool bsums = fsums == 1;
  sc.cur_bitsums = bsums;
  if (fsums == 2) {  // msm_finish: slot 0 + kSeg29 * sum_b 2^b slot_{1+b}
    sc.cur_nbits = p.nslots29 - 1;
    sc.cur_seglen = kSeg29;
  }
  const bool phases = sc.prof && sc.prof_phases;
  if (sc.prof && !sc.ev[0])
    for (auto& e : sc.ev) NZ_HIP(hipEventCreate(&e));
  auto mark = [&](int i) {
    if (phases) NZ_HIP(hipEventRecord(sc.ev[i], st));
  };
  mark(0);
  const bool bins = table && p.c >= 16 && p.c <= 20 && !use_library_sort() && sc.bin_counts.p;
  if (bins) {  // hand-written bucketing (see msm_bin_hist_kernel)
    const uint32_t ntiles = (uint32_t)((n + kTileScalars - 1) / kTileScalars);
    uint32_t* tail = sc.bin_counts.p + (size_t)256 * ntiles;
    const int m = mdig;
    auto run_bins = [&](auto cc) {
      constexpr int C = decltype(cc)::value;
      using Lo = typename BinKeys<C>::Lo;
      Lo* lo2 = (Lo*)sc.keys_out.p;
      hipLaunchKernelGGL(msm_bin_hist_kernel<C>, dim3(ntiles), dim3(kBinThreads), 0, st, scalars, n, m,
                         sc.bin_counts.p, ntiles);
      NZ_HIP(hipGetLastError());
      mark(1);
      hipLaunchKernelGGL(msm_bin_rowscan_kernel, dim3(256), dim3(256), 0, st, sc.bin_counts.p, ntiles, tail);
      hipLaunchKernelGGL(msm_bin_scatter_kernel<C>, dim3(ntiles), dim3(kBinThreads), 0, st, scalars, n, m,
                         table->stride, sc.bin_counts.p, ntiles, lo2, sc.vals_mid.p);
      NZ_HIP(hipGetLastError());
      mark(2);
      constexpr int LO = BinKeys<C>::LO;
      if (!lo_split()) {
        hipLaunchKernelGGL(msm_bucket_lo_kernel<LO>, dim3(256), dim3(kLoThreads), 0, st, (const Lo*)lo2,
                           sc.vals_mid.p, sc.bin_counts.p, ntiles, p.nkeys, sc.offsets.p, sc.sorted.p, sc.large.p);
        NZ_HIP(hipGetLastError());
        return;
      }
      const dim3 igrid((unsigned)lo_items_bound(p.entries));
      hipLaunchKernelGGL((lo_agg() ? msm_lo_count_kernel<LO, true> : msm_lo_count_kernel<LO, false>), igrid,
                         dim3(kLoThreads), 0, st, (const Lo*)lo2, sc.bin_counts.p, ntiles, sc.lo_seg.p);
      NZ_HIP(hipGetLastError());
      hipLaunchKernelGGL(msm_lo_scan_kernel<LO>, dim3(256), dim3(kLoThreads), 0, st, sc.bin_counts.p, ntiles,
                         sc.lo_seg.p, p.nkeys, sc.offsets.p, sc.large.p);
      NZ_HIP(hipGetLastError());
      hipLaunchKernelGGL((lo_agg() ? msm_lo_scatter_kernel<LO, true> : msm_lo_scatter_kernel<LO, false>), igrid,
                         dim3(kLoThreads), 0, st, (const Lo*)lo2, sc.vals_mid.p, sc.bin_counts.p, ntiles,
                         (const uint32_t*)sc.lo_seg.p, sc.sorted.p);
      NZ_HIP(hipGetLastError());
    };
    switch (p.c) {
      case 16: run_bins(std::integral_constant<int, 16>()); break;
      case 17: run_bins(std::integral_constant<int, 17>()); break;
      case 18: run_bins(std::integral_constant<int, 18>()); break;
      case 19: run_bins(std::integral_constant<int, 19>()); break;
      default: run_bins(std::integral_constant<int, 20>()); break;
    }
  } else {
    keys_dispatch(p.c, scalars, n, mdig, table, sc, st);
    mark(1);
  }
  size_t tmp = sc.sort_tmp_bytes;
  const dim3 ogrid(grid_for((size_t)p.nkeys + 1, kMsmThreads, 1u << 30));
  if (bins) {
    // offsets written by msm_lo_scan_kernel
  } else if (table && p.nkeys <= 65536) {  // 16-bit keys, no sentinel (see msm_keys_kernel)
    int end_bit = 0;
    while ((1u << end_bit) < p.nkeys) end_bit++;
    radix_sort(sc.sort_tmp.p, tmp, (const uint16_t*)sc.keys_in.p, (uint16_t*)sc.keys_out.p, sc.vals_in.p,
               sc.sorted.p, p.entries, end_bit, st);
    mark(2);
    hipLaunchKernelGGL(msm_offsets_kernel<uint16_t>, ogrid, dim3(kMsmThreads), 0, st, (const uint16_t*)sc.keys_out.p,
                       p.entries, p.nkeys, sc.offsets.p);
  } else {
    int end_bit = 1;
    while ((1u << end_bit) <= p.nkeys) end_bit++;
    radix_sort(sc.sort_tmp.p, tmp, sc.keys_in.p, sc.keys_out.p, sc.vals_in.p, sc.sorted.p, p.entries, end_bit, st);
    mark(2);
    hipLaunchKernelGGL(msm_offsets_kernel<uint32_t>, ogrid, dim3(kMsmThreads), 0, st, sc.keys_out.p, p.entries,
                       p.nkeys, sc.offsets.p);
  }
  NZ_HIP(hipGetLastError());
  if (sc.prof) NZ_HIP(hipEventRecord(sc.ev[3], st));
  // pairing rounds (fixed base): each halves every bucket's run of entries
  const int rounds = table ? pair_rounds_for(p.entries, p.nkeys) : 0;
  const uint32_t* acc_off = sc.offsets.p;
  const G1Affine* acc_src = gather;
  size_t acc_entries = p.entries;
  for (int r = 0; r < rounds; r++) {
    uint32_t* noff = sc.pair_off[r & 1].p;
    G1Affine* dst = sc.pair_pts[r & 1].p;
    const size_t bound = pair_bound(acc_entries, p.nkeys);
    if (!noff || bound > sc.pair_pts[r & 1].n || pair_grid(bound) * kPairThreads * kPairPer * 9 > sc.pair_pre.n ||
        p.nkeys + 1 > sc.pair_off[r & 1].n)
      throw Error(NZCB_ERR_ARG, "msm scratch was not sized for the pairing rounds");
    hipLaunchKernelGGL(msm_pair_offsets_kernel, dim3(1), dim3(1024), 0, st, acc_off, p.nkeys, noff);
    NZ_HIP(hipGetLastError());
    const dim3 pgrid((uint32_t)pair_grid(bound));
    if (r == 0)
      hipLaunchKernelGGL(msm_pair29_kernel<true>, pgrid, dim3(kPairThreads), 0, st, acc_src, sc.sorted.p, acc_off,
                         noff, p.nkeys, sc.pair_pre.p, dst);
    else
      hipLaunchKernelGGL(msm_pair29_kernel<false>, pgrid, dim3(kPairThreads), 0, st, acc_src, sc.sorted.p, acc_off,
                         noff, p.nkeys, sc.pair_pre.p, dst);
    NZ_HIP(hipGetLastError());
    acc_off = noff;
    acc_src = dst;
    acc_entries = bound;
  }
  const uint32_t chunk = chunk_for(acc_entries);
  const size_t nthreads = (acc_entries + chunk - 1) / chunk;
  // waves per SIMD the accumulation is compiled for (NZCB_ACC29_WAVES = 2..4 for A/B
  // runs). 3 (<= 168 VGPRs): at 4 (<= 128) the prefetched next point spilled to scratch,
  // 80 B stored and reloaded per entry (WRITE_SIZE 2.5 GB per launch); 2.55 -> 2.29 ms
  static const int acc_waves = [] {
    const char* e = std::getenv("NZCB_ACC29_WAVES");
    const int w = e ? std::atoi(e) : 3;
    return w >= 2 && w <= 4 ? w : 3;
  }();
  const dim3 agrid(grid_for(nthreads, kMsmThreads, 1u << 30));
  if (table) {
    if (!sc.buckets29.p) throw Error(NZCB_ERR_ARG, "msm scratch was not sized for the fixed-base schedule");
    if (rounds)
      hipLaunchKernelGGL((msm_accumulate29_kernel<3, true>), agrid, dim3(kMsmThreads), 0, st, chunk, acc_src,
                         sc.sorted.p, acc_off, p.nkeys, nthreads, sc.buckets29.p, sc.carry_own29.p,
                         sc.carry_cont29.p);
    else if (chunk == kChunk && acc_dma())
      hipLaunchKernelGGL(msm_accumulate29_dma_kernel, agrid, dim3(kMsmThreads), 0, st, gather, sc.sorted.p,
                         sc.offsets.p, p.nkeys, nthreads, sc.buckets29.p, sc.carry_own29.p, sc.carry_cont29.p);
    else if (chunk == kChunk && acc_waves == 3 && lds_indices())
      hipLaunchKernelGGL((!paired_products() ? msm_accumulate29_kernel<3, false, true, false>
                          : acc_aff()        ? msm_accumulate29_kernel<3, false, true, true, true>
                                             : msm_accumulate29_kernel<3, false, true, true>),
                         agrid, dim3(kMsmThreads), 0, st, chunk, gather, sc.sorted.p, sc.offsets.p, p.nkeys, nthreads,
                         sc.buckets29.p, sc.carry_own29.p, sc.carry_cont29.p);
    else
      hipLaunchKernelGGL(acc_waves == 4 ? msm_accumulate29_kernel<4>
                                        : (acc_waves == 2 ? msm_accumulate29_kernel<2> : msm_accumulate29_kernel<3>),
                         agrid,
                         dim3(kMsmThreads), 0, st, chunk, gather, sc.sorted.p, sc.offsets.p, p.nkeys, nthreads,
                         sc.buckets29.p, sc.carry_own29.p, sc.carry_cont29.p);
  } else {
    hipLaunchKernelGGL(msm_accumulate_kernel, agrid, dim3(kMsmThreads), 0, st, chunk, gather, sc.sorted.p, sc.offsets.p,
                       p.nkeys, nthreads, sc.buckets.p, sc.carry_own.p, sc.carry_cont.p);
  }
  NZ_HIP(hipGetLastError());
  if (sc.prof) NZ_HIP(hipEventRecord(sc.ev[4], st));
  if (!bins) NZ_HIP(hipMemsetAsync(sc.large.p, 0, sizeof(uint32_t), st));  // bins: zeroed by msm_lo_scan_kernel
  const dim3 fgrid(grid_for(p.nkeys, kMsmThreads, 1u << 30));
  if (table) {
    Xyzz29* out29 = fsums ? sc.buckets29.p : nullptr;
    if (out29 && fin_lanes() == 4)
      hipLaunchKernelGGL(msm_finalize29_kernel, dim3(grid_for((size_t)p.nkeys * 4, kMsmThreads, 1u << 30)),
                         dim3(kMsmThreads), 0, st, chunk, acc_off, p.nkeys, (const Xyzz29*)sc.carry_own29.p,
                         (const Xyzz29*)sc.carry_cont29.p, sc.large.p, out29);
    else
      hipLaunchKernelGGL(msm_bucket_finalize_kernel<Xyzz29>, fgrid, dim3(kMsmThreads), 0, st, chunk, acc_off,
                         p.nkeys, seq_span29(), (const Xyzz29*)sc.buckets29.p, (const Xyzz29*)sc.carry_own29.p,
                         (const Xyzz29*)sc.carry_cont29.p, sc.buckets.p, sc.large.p, out29);
    NZ_HIP(hipGetLastError());
    hipLaunchKernelGGL(msm_large_scan_kernel, dim3(1), dim3(1024), 0, st, chunk, acc_off, sc.large.p,
                       sc.large_off.p);
    NZ_HIP(hipGetLastError());
    hipLaunchKernelGGL(msm_large_piece29_kernel, dim3(kLargePieceBlocks), dim3(kSumThreads), 0, st, chunk, acc_off,
                       sc.large.p, sc.large_off.p, (const Xyzz29*)sc.carry_own29.p,
                       (const Xyzz29*)sc.carry_cont29.p, sc.large_part.p);
    NZ_HIP(hipGetLastError());
    hipLaunchKernelGGL(msm_large_final29_kernel, dim3(kLargeFinalBlocks), dim3(kLargeFinalThreads), 0, st, sc.large.p,
                       sc.large_off.p, sc.large_part.p, sc.buckets.p, out29);
  } else {
    hipLaunchKernelGGL(msm_bucket_finalize_kernel<G1xyzz>, fgrid, dim3(kMsmThreads), 0, st, chunk, sc.offsets.p, p.nkeys,
                       kSeqSpan29, (const G1xyzz*)nullptr, (const G1xyzz*)sc.carry_own.p, (const G1xyzz*)sc.carry_cont.p,
                       sc.buckets.p, sc.large.p, (Xyzz29*)nullptr);
    NZ_HIP(hipGetLastError());
    hipLaunchKernelGGL(msm_bucket_large_kernel<G1xyzz>, dim3(kLargeBlocks), dim3(kSumThreads), 0, st, chunk,
                       sc.offsets.p,
                       sc.large.p, (const G1xyzz*)sc.carry_own.p, (const G1xyzz*)sc.carry_cont.p, sc.buckets.p);
  }
  NZ_HIP(hipGetLastError());
  mark(5);
  if (fsums == 2) {
    hipLaunchKernelGGL(msm_seg29_kernel, dim3(grid_for((size_t)p.nseg29, kMsmThreads, 1u << 30)), dim3(kMsmThreads),
                       0, st, (const Xyzz29*)sc.buckets29.p, acc_off, (uint32_t)p.nseg29, sc.seg_tot29.p,
                       sc.seg_run29.p);
    NZ_HIP(hipGetLastError());
    mark(6);
    hipLaunchKernelGGL(msm_segsums29_kernel, dim3(p.nslots29 * p.sparts29), dim3(kSumThreads), 0, st,
                       (const Xyzz29*)sc.seg_tot29.p, (const Xyzz29*)sc.seg_run29.p, p.nseg29, p.sparts29,
                       sc.parts29.p);
    NZ_HIP(hipGetLastError());
    hipLaunchKernelGGL(msm_parts29_kernel, dim3(p.nslots29), dim3(kPartThreads), 0, st, (const Xyzz29*)sc.parts29.p,
                       p.sparts29, sc.win.p);
    NZ_HIP(hipGetLastError());
    mark(7);
    NZ_HIP(hipMemcpyAsync(sc.host_win, sc.win.p, (size_t)p.nslots29 * sizeof(G1xyzz), hipMemcpyDeviceToHost, st));
    NZ_HIP(hipEventRecord(sc.done, st));
    return;
  }
  if (bsums) {
    mark(6);
    hipLaunchKernelGGL(msm_bitsums29_kernel, dim3((p.lb + 1) * p.bparts), dim3(kSumThreads), 0, st,
                       (const Xyzz29*)sc.buckets29.p, acc_off, p.lb, p.bparts, sc.parts29.p);
    NZ_HIP(hipGetLastError());
    hipLaunchKernelGGL(msm_parts29_kernel, dim3(p.lb + 1), dim3(kPartThreads), 0, st, (const Xyzz29*)sc.parts29.p,
                       p.bparts, sc.win.p);
    NZ_HIP(hipGetLastError());
    mark(7);
    NZ_HIP(hipMemcpyAsync(sc.host_win, sc.win.p, (size_t)(p.lb + 1) * sizeof(G1xyzz), hipMemcpyDeviceToHost, st));
    NZ_HIP(hipEventRecord(sc.done, st));
    return;
  }
  hipLaunchKernelGGL(msm_bucket_reduce_kernel, dim3(grid_for((size_t)p.nsets * p.nseg, kMsmThreads, 1u << 30)),
                     dim3(kMsmThreads), 0, st, sc.buckets.p, sc.offsets.p, (int)p.nb, p.seglen, p.nseg, p.nsets,
                     sc.seg_tot.p, sc.seg_run.p);
  NZ_HIP(hipGetLastError());
  mark(6);
  hipLaunchKernelGGL(msm_sums_kernel, dim3(p.nsets * p.nslots * p.nparts), dim3(kSumThreads), 0, st, sc.seg_tot.p,
                     sc.seg_run.p, p.nseg, p.nslots, p.nparts, sc.parts.p);
  NZ_HIP(hipGetLastError());
  hipLaunchKernelGGL(msm_parts_kernel, dim3(p.nsets * p.nslots), dim3(kPartThreads), 0, st, sc.parts.p, p.nparts,
                     sc.win.p);
  NZ_HIP(hipGetLastError());
  mark(7);
  NZ_HIP(hipMemcpyAsync(sc.host_win, sc.win.p, (size_t)p.nsets * p.nslots * sizeof(G1xyzz), hipMemcpyDeviceToHost,
                        st));
  NZ_HIP(hipEventRecord(sc.done, st));
}

G1xyzz msm_finish(MsmScratch& sc, hipStream_t st) {
  if (sc.cur_n == 0) return G1xyzz::inf();
  // the window sums' copy, not the whole stream: work queued on the stream after the MSM
  // (the prover's A/B/C interpolations follow C's commitment on its stream) runs on
  NZ_HIP(hipEventSynchronize(sc.done));
  const int c = sc.cur_c, nsets = sc.cur_nsets, nslots = sc.cur_nbits + 1;
  if (sc.prof) {
    float t = 0;
    NZ_HIP(hipEventElapsedTime(&t, sc.ev[3], sc.ev[4]));
    uint32_t total = 0;
    NZ_HIP(hipMemcpyAsync(&total, sc.offsets.p + sc.cur_nkeys, 4, hipMemcpyDeviceToHost, st));
    NZ_HIP(hipStreamSynchronize(st));
    sc.prof_ms += t;
    sc.prof_launches++;
    sc.prof_points += sc.cur_n;
    sc.prof_entries += total;
    if (sc.prof_phases) {
      // keys, sort, offsets, accumulate, finalize, reduce, sums
      for (int i = 0; i < 7; i++) {
        float ms = 0;
        NZ_HIP(hipEventElapsedTime(&ms, sc.ev[i], sc.ev[i + 1]));
        sc.phase_ms[i] += ms;
      }
    }
  }
  if (sc.cur_bitsums) {  // sum_b 2^b S_b over the lb + 1 = c bit slots (msm_bitsums29_kernel)
    G1xyzz acc = G1xyzz::inf();
    for (int b = c - 1; b >= 0; b--) {
      acc = xyzz_dbl(acc);
      acc = xyzz_add(acc, sc.host_win[b]);
    }
    return acc;
  }
  int lg_seg = 0;
  while ((1 << lg_seg) < sc.cur_seglen) lg_seg++;
  G1xyzz res = G1xyzz::inf();
  for (int w = nsets - 1; w >= 0; w--) {
    const G1xyzz* s = sc.host_win + (size_t)w * nslots;
    // sum_g g * run_g = sum_b 2^b R_b  (Horner over the bits), times the segment length
    G1xyzz acc = G1xyzz::inf();
    for (int b = nslots - 2; b >= 0; b--) {
      acc = xyzz_dbl(acc);
      acc = xyzz_add(acc, s[1 + b]);
    }
    for (int i = 0; i < lg_seg; i++) acc = xyzz_dbl(acc);
    const G1xyzz W = xyzz_add(acc, s[0]);
    if (nsets > 1)
      for (int i = 0; i < c; i++) res = xyzz_dbl(res);
    res = xyzz_add(res, W);
  }
  return res;
}

}  // namespace nzcb
