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
//    (key = window * 2^(c-1) + |digit| - 1), rocPRIM radix sort, 8x32 XYZZ buckets,
//    host Horner over the windows;
//  * fixed-base (the prover's PTau and Lagrange tables): a table of shifted bases
//    2^(c*w) * B_i (MsmBaseTable) turns the windows into ONE set of 2^(c-1) buckets (key =
//    |digit| - 1, value = row w of the table) and a single bucket reduction, all in the
//    carry-free 9 x 29-bit radix of csrc/f29.h (table stored Montgomery-261).
//
// Fixed-base pipeline (one stream, no host sync until the slot sums):
//  1. bucketing:  counting sort by the bucket index, hand-written (msm_bin_* / msm_lo_*)
//  2. accumulate: thread per fixed 48-entry chunk of the bucketed stream (load balance
//                 independent of the digits): XYZZ mixed adds of the gathered table points;
//                 bucket runs inside one chunk are written directly, runs crossing a chunk
//                 edge go to per-chunk carries
//  3. finalize:   thread per bucket spanning chunks adds its carries (long runs: pieces
//                 summed by workgroups)
//  4. window sum: sum_k (k + 1) B_k by the two-dimensional reduction (msm_tile29_kernel):
//                 row and column plain sums, then bit-slot sums over the lines
//  5. host:       the slots combined by doublings
#include "msm.h"

#include "f29.h"

#include <chrono>
#include <cstdlib>
#include <type_traits>
#include <rocprim/rocprim.hpp>
#include <rocprofiler-sdk-roctx/roctx.h>

namespace nzcb {

static constexpr int kMsmThreads = 256;

// Wave issue priority of the latency-bound MSM kernels (the fixed-base finalize, carry trees and
// window sums, the sparse schedule's accumulation): under several proof lanes their few waves
// share SIMDs with VALU-bound waves (other lanes' bucket accumulations, NTT passes) and got a
// fraction of the issue slots, which stretched every dependent addition. s_setprio raises
// them over the co-resident waves in the SIMD's arbitration (0 = off).
#ifndef NZ_TAIL_PRIO
#define NZ_TAIL_PRIO 0
#endif
__device__ __forceinline__ void tail_prio() {
  if constexpr (NZ_TAIL_PRIO > 0) __builtin_amdgcn_s_setprio(NZ_TAIL_PRIO);
}

// Onesweep with a chosen digit width (generic schedule): the 20-bit keys take 2 passes of
// 10 bits instead of 3 with the library's 8-bit default for gfx950 (2^21: 0.55 vs 0.69 ms)
using SortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 16>, rocprim::kernel_config<1024, 16>, 10,
                                        rocprim::block_radix_rank_algorithm::match>>;

static void radix_sort(void* tmp, size_t& tmp_bytes, const uint32_t* kin, uint32_t* kout, const uint32_t* vin,
                       uint32_t* vout, size_t m, int end_bit, hipStream_t st) {
  NZ_HIP(rocprim::radix_sort_pairs<SortConfig>(tmp, tmp_bytes, kin, kout, vin, vout, m, 0, end_bit, st));
}

// entries per accumulation thread, up to 2^26 entries: 48 cuts the carries the finalize
// adds by a third against 32 (same box: bench 32.5 -> 32.9 proofs/s; isolated
// accumulate + finalize 2.8 ms for 32, 40 and 48, 2.9 ms for 64, whose 1.9 rounds of
// waves leave a tail)
static constexpr uint32_t kChunk = 48;

// Entries per accumulation thread: kChunk up to 2^26 entries, then doubled so the grid
// stays ~2^19-2^20 threads and a bucket spans ~10 chunks at every size (at 2^24 points a
// fixed 32-entry chunk left ~120 carries per bucket and the finalize took 360 ms).
static uint32_t chunk_for(size_t entries) {
  uint32_t c = kChunk;
  while (entries / c > (size_t(1) << 20)) c *= 2;
  return c;
}
static constexpr int kSegLen = 8;
static constexpr int kSumThreads = 256;  // level-1 sums: block size
static constexpr int kSumPer = 4;        // level-1 sums: sequential adds per thread
static constexpr int kPartThreads = 64;  // level-2 sums: block size
static constexpr uint32_t kSeqSpan = 64;  // finalize: longest carry run summed by one thread
// the same for the fixed-base (radix 2^29) carries: at 2^21 random scalars a bucket spans
// ~11 chunks at c = 17, ~2 at c = 20; the Lagrange-basis commitments' skewed digits leave a
// few hundred buckets with 17..1000s of carries, and a thread walking 64 of them
// sequentially was the finalize's long pole (0.8 ms per launch, round 1)
static constexpr uint32_t kSeqSpan29 = 16;
static constexpr int kLargeBlocks = 32;  // finalize: workgroups for the longer runs
// fixed base: workgroups over the pieces of the longer runs, and over their buckets (grid-
// stride; random scalars list none, and under 5 proof lanes every launched workgroup waits
// for a CU slot first, so the dense tables' grids are kept small)
static constexpr int kLargePieceBlocks = 128;
static constexpr int kLargeFinalBlocks = 128;

// Sparse tables (MsmBaseTable::sparse: the Lagrange basis, whose A, B, C scalars are mostly
// 0, 1 and bytes; round 6). Their few entries (~0.7-1.5 per scalar against 13 for random
// ones) left most of the chip idle behind 48-entry chains, and |digit| = 1 puts ~40 % of the
// entries into one bucket whose carries went through ~80 dependent additions (48 in the
// chain, 16 in the finalize, 12 in the pieces, ~7 in their sum). The MSM's time is its
// depth in dependent EC additions (~15-20 us each with a wave or two per SIMD), so:
//  * the chunk is derived on the device from the bucketed entry count M: ceil(M / 2^18)
//    entries per thread, clamped to [kDynMin, kChunk] (every kernel that maps stream
//    positions to chunks computes the same dyn_chunk(M));
//  * the finalize sums runs of at most kSeqSpanSparse + 1 carries per lane;
//  * longer runs are cut into pieces of kPieceCarries summed by log-depth LDS trees, and a
//    bucket's pieces by another tree: ceil(log2(carries)) + 1 dependent additions.
static constexpr uint32_t kDynThreads = 1u << 18;
static constexpr uint32_t kDynMin = 8;
static constexpr uint32_t kSeqSpanSparse = 3;
static constexpr int kSparsePieceBlocks = 2048;
static constexpr int kSparseFinalBlocks = 512;
__host__ __device__ __forceinline__ uint32_t dyn_chunk(uint32_t m) {
  const uint32_t c = (m + kDynThreads - 1) / kDynThreads;
  return c < kDynMin ? kDynMin : c > kChunk ? kChunk : c;
}
// the most accumulation threads dyn_chunk gives for any count M <= entries: ceil(M / chunk)
// <= 2^18 while the chunk is unclamped or kDynMin (M <= kDynMin 2^18), else ceil(M / kChunk)
static size_t dyn_threads_bound(size_t entries) {
  const size_t lo = std::min<size_t>(kDynThreads, (entries + kDynMin - 1) / kDynMin);
  return std::max<size_t>(lo, (entries + kChunk - 1) / kChunk);
}

// Fixed-base window of the PTau tables: c = 20 bits (13 table rows, 2^19 buckets, 13
// entries per random scalar) since round 5, when the window sum's first level became the
// LDS-free strip kernel (msm_strips29_kernel): same box, bench.py --steps 200, 42.50 / 42.36
// proofs/s at c = 20 against 41.45 / 41.23 at c = 17 (profiles/r5_window_ab.txt); until round 4
// c = 17 (15 rows, 2^16 buckets) won, its 55 KB-LDS tile kernel at 2^19 buckets costing more
// than the 13 % fewer entries saved. NZCB_FB_WINDOW = 16..20 selects another.
static constexpr int kFbWindow = 20;
int fixed_base_window() {
  static const int c = [] {
    const char* e = std::getenv("NZCB_FB_WINDOW");
    const int v = e ? std::atoi(e) : kFbWindow;
    return (v >= 16 && v <= 20) ? v : kFbWindow;
  }();
  return c;
}

// the Lagrange-basis table's window: its small scalars make few entries, which do not pay
// for a larger bucket set (round 5, same box: c = 20 here lost 1.2-1.5 % of the bench,
// profiles/r5_chunk_key_lw20_ab.txt)
#ifndef NZ_LAGRANGE_WINDOW
#define NZ_LAGRANGE_WINDOW 17
#endif
int lagrange_window() { return NZ_LAGRANGE_WINDOW; }
bool lagrange_sparse() {
  static const bool v = [] {
    const char* e = std::getenv("NZCB_SPARSE");
    return e && std::atoi(e) != 0;
  }();
  return v;
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

#ifdef NZCB_MSM_STATS
template <class F>
static void for_each_digit_host(const Fr& s, int C, F&& f) {
  const int NW = (255 + C - 1) / C;
  const uint32_t MASK = (1u << C) - 1u, HALF = 1u << (C - 1);
  uint32_t carry = 0;
  for (int w = 0; w < NW; w++) {
    const int bit = w * C, limb = bit >> 5, sh = bit & 31;
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
#endif

// generic schedule: key = w * NB + bucket, value = i | sign << 31; zero digits a sentinel
// key that sorts after every bucket
template <int C>
__global__ void __launch_bounds__(kMsmThreads)
msm_keys_kernel(const Fr* __restrict__ scalars, size_t n, int mont, uint32_t* __restrict__ keys,
                uint32_t* __restrict__ vals) {
  constexpr int NW = (255 + C - 1) / C;
  constexpr uint32_t NB = 1u << (C - 1);
  constexpr uint32_t SENTINEL = NW * NB;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    Fr s = scalars[i];
    if (mont) s = from_mont_fr29(s);
    uint32_t k[NW];
#pragma unroll
    for (int w = 0; w < NW; w++) k[w] = SENTINEL;
    uint32_t sg[NW];
#pragma unroll
    for (int w = 0; w < NW; w++) sg[w] = 0;
    for_each_digit<C>(s, [&](int w, uint32_t b, uint32_t sign) {
      k[w] = (uint32_t)w * NB + b;
      sg[w] = sign << 31;
    });
#pragma unroll
    for (int w = 0; w < NW; w++) {
      keys[(size_t)w * n + i] = k[w];
      vals[(size_t)w * n + i] = (uint32_t)i | sg[w];
    }
  }
}

// ---- fixed-base bucketing, replacing a library radix sort -----------------------------
// Entries (one per scalar and nonzero window digit) are grouped by bucket in two counting
// passes, over the bucket index's high byte and then its low bits, reduce-then-scan, with
// every counter in LDS or fully written (no look-back spinning, no fills):
//   1. msm_bin_hist_kernel    per tile of 512 scalars: the digits, and the histogram of
//                             the keys' high byte -> counts[hi][tile]
//   2. msm_bin_rowscan_kernel per high byte: exclusive scan over the tiles and the row
//                             total (consumers scan the 256 totals for the region starts)
//   3. msm_bin_scatter_kernel per tile: the digits again (32 B read per scalar instead of
//                             the entries), ranked in LDS by high byte, then written
//                             out run by run (coalesced) into the high-byte regions: the
//                             value and the key's low bits
//   4. msm_lo_*_kernel        per high byte (split into segments, see below): low-bits
//                             histogram of its region, local scan -> the bucket offsets,
//                             scatter
// Order inside a bucket is whatever the LDS atomics give: the accumulation adds the
// bucket's points in any order and the sum is the same point.
// 256- and 512-thread workgroups with modest LDS: under 5 proof lanes these kernels share
// the CUs with the accumulation's waves, and a 1024-thread or 95 KB-LDS workgroup waits
// for a whole CU to drain (measured: 5.3 ms average scatter launch in the pipeline)
static constexpr int kBinThreads = 256;
static constexpr int kBinPer = 2;                                  // scalars per thread and tile
static constexpr uint32_t kTileScalars = kBinThreads * kBinPer;    // 512
static constexpr int kLoThreads = 512;

// the (key, value) of every window of scalar i; bit w of the result is set for the
// windows with a nonzero digit (zero digits make no entry: a scalar of b bits costs about
// b / C entries, which the Lagrange-basis commitments of small witness values rely on)
// digit-pass flags (the `mont` argument of the bucketing kernels)
static constexpr int kDigMont = 1;     // scalars in Montgomery form: convert first
static constexpr int kDigMinForm = 2;  // bucket min(s, r - s) (scalar_min_form)

// Signed scalars (round 6): s and r - s reach the same point with the base negated (every
// base has order r), and the fixed-base schedule buckets whichever of the two is smaller, the
// negation riding in every entry's sign bit. Random scalars lose nothing (their 13 windows stay
// occupied); the Lagrange-basis A, B, C values, of which 13-29 % are small negatives r - k
// (15 nonzero 17-bit digits as they stand, one as k), fall from 21.7 M to 4.7 M bucket
// entries per proof (nzcp_live, profiles/r6_abc_scalars.txt). The prover's folded PTau
// tables (random scalars: the compare and negation bought nothing and cost 0.05 G VALU
// instructions per proof) skip it; every unfolded table (Lagrange, split ranges, engine)
// takes it. Values >= r (never produced) are left as they are. Returns 1 when s was
// replaced by r - s.
__device__ __forceinline__ uint32_t scalar_min_form(Fr& s) {
  constexpr uint32_t H[8] = {0xf8000000u, 0xa1f0fac9u, 0x3cdcb848u, 0x9419f424u,
                             0x40c0ac2eu, 0xdc2822dbu, 0x7098d014u, 0x18322739u};  // (r - 1) / 2
  bool gt = false, eq = true, lt_r = false, eq_r = true;
#pragma unroll
  for (int l = 7; l >= 0; l--) {
    gt = gt || (eq && s.v[l] > H[l]);
    eq = eq && s.v[l] == H[l];
    lt_r = lt_r || (eq_r && s.v[l] < FrParams::P[l]);
    eq_r = eq_r && s.v[l] == FrParams::P[l];
  }
  if (!(gt && lt_r)) return 0u;
  s = neg(s);
  return 1u;
}

template <int C, int NW>
__device__ __forceinline__ uint32_t bin_entries(const Fr* __restrict__ scalars, size_t i, int mont, size_t stride,
                                                uint32_t (&kk)[NW], uint32_t (&vv)[NW]) {
  Fr s = scalars[i];
  if (mont & kDigMont) s = from_mont_fr29(s);
  const uint32_t flip = (mont & kDigMinForm) ? scalar_min_form(s) : 0u;
  uint32_t live = 0;
#pragma unroll
  for (int w = 0; w < NW; w++) {
    kk[w] = 0;
    vv[w] = 0;
  }
  for_each_digit<C>(s, [&](int w, uint32_t b, uint32_t sign) {
    kk[w] = b;
    vv[w] = (uint32_t)((size_t)w * stride + i) | ((sign ^ flip) << 31);
    live |= 1u << w;
  });
  return live;
}

// bucket index bits below the high byte, for KB-bit bucket keys: 8 up to 16-bit keys (c <= 17),
// KB - 8 above (c = 20: 19-bit keys, 256 high-byte regions of 2048 buckets; three c = 17 bucket
// sets: 18-bit keys)
template <int KB> struct BinKeys {
  static constexpr int LO = KB - 8 > 8 ? KB - 8 : 8;
  using Lo = typename std::conditional<LO <= 8, uint8_t, uint16_t>::type;      // low part, per entry
  using Full = typename std::conditional<KB <= 16, uint16_t, uint32_t>::type;  // whole key, in LDS
};

// Several MSMs over one table in one schedule (round 6: A, B and C over the Lagrange basis):
// set s's scalars are tiles [s tps, (s + 1) tps) of the bucketing grid and its buckets keys
// [s nb, (s + 1) nb), so one sort, one accumulation and one carry reduction serve all of them,
// and the window sums run per set. One set: tps = all tiles.
static constexpr int kMaxSets = 3;
struct BinSets {
  const Fr* p[kMaxSets];
  uint32_t tps;  // bucketing tiles per set
  uint32_t nb;   // buckets per set
};

template <int C, int KB>
__global__ void __launch_bounds__(kBinThreads)
msm_bin_hist_kernel(BinSets sets, size_t n, int mont, uint32_t* __restrict__ counts, uint32_t ntiles) {
  constexpr int NW = (255 + C - 1) / C;
  constexpr int LO = BinKeys<KB>::LO;
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t set = blockIdx.x / sets.tps, lt = blockIdx.x - set * sets.tps;
  const Fr* __restrict__ scalars = sets.p[set];
  const uint32_t kbase = set * sets.nb;
#pragma unroll
  for (int j = 0; j < kBinPer; j++) {
    const size_t i = (size_t)lt * kTileScalars + (size_t)j * kBinThreads + threadIdx.x;
    if (i < n) {
      uint32_t kk[NW], vv[NW];
      const uint32_t live = bin_entries<C, NW>(scalars, i, mont, 0, kk, vv);
#pragma unroll
      for (int w = 0; w < NW; w++)
        if ((live >> w) & 1u) atomicAdd(&h[(kk[w] + kbase) >> LO], 1u);
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

template <int C, int KB>
__global__ void __launch_bounds__(kBinThreads)
msm_bin_scatter_kernel(BinSets sets, size_t n, int mont, size_t stride, const uint32_t* __restrict__ counts,
                       uint32_t ntiles, typename BinKeys<KB>::Lo* __restrict__ lo2, uint32_t* __restrict__ vals2) {
  constexpr int NW = (255 + C - 1) / C;
  constexpr int TE = kTileScalars * NW;  // entries per tile, at most
  constexpr int LO = BinKeys<KB>::LO;
  __shared__ uint32_t lcount[256], lstart[256], gbase[256];
  __shared__ uint32_t lval[TE];
  __shared__ typename BinKeys<KB>::Full lkey[TE];
  const uint32_t set = blockIdx.x / sets.tps, lt = blockIdx.x - set * sets.tps;
  const Fr* __restrict__ scalars = sets.p[set];
  const uint32_t kbase = set * sets.nb;
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
    const size_t i = (size_t)lt * kTileScalars + (size_t)j * kBinThreads + threadIdx.x;
    live[j] = 0;
    if (i < n) {
      live[j] = bin_entries<C, NW>(scalars, i, mont, stride, kk[j], vv[j]);
#pragma unroll
      for (int w = 0; w < NW; w++) {
        kk[j][w] += kbase;
        if ((live[j] >> w) & 1u) rk[j][w] = atomicAdd(&lcount[kk[j][w] >> LO], 1u);
      }
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
        lkey[q] = (typename BinKeys<KB>::Full)kk[j][w];
        lval[q] = vv[j][w];
      }
    }
  }
  __syncthreads();
  for (uint32_t q = threadIdx.x; q < total; q += kBinThreads) {  // runs of one high byte: coalesced
    const uint32_t key = lkey[q], hb = key >> LO;
    const uint32_t pos = gbase[hb] + (q - lstart[hb]);
    lo2[pos] = (typename BinKeys<KB>::Lo)(key & ((1u << LO) - 1u));
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
// in round 2; 0.1 ms for random scalars):
//   a. msm_lo_count_kernel   per item: low-index histogram of its segment -> segoff[item][.]
//   b. msm_lo_scan_kernel    per region: exclusive scan over its items per bucket, the
//                            bucket offsets (scan over the buckets), segoff += bucket offset
//   c. msm_lo_scatter_kernel per item: ranked in LDS chunk by chunk, written run by run
// Plain LDS atomics: with regions cut into kLoSeg segments a hot bucket's same-address
// conflicts cost ~15 us per workgroup (wave-aggregated atomics cost ~10 instructions per
// entry on every entry of every MSM, round 3)
static constexpr uint32_t kLoSeg = 32768;
static constexpr uint32_t kLoU = 8;  // entries per thread and chunk

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

template <int LO>
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
    for (uint32_t u = 0; u < kLoU; u++)
      if (k8[u] < NL) atomicAdd(&h[k8[u]], 1u);
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

// c > 17 (LO = 11: 2048 buckets per high-byte region): 1024 threads ranking 16384-entry
// chunks in LDS (122 KB, one workgroup per CU) instead of 512 x 8. A 4096-entry chunk left
// runs of ~2 entries per bucket, so the coalesced write-out degenerated into 8-byte pieces;
// at 16384 they average 8 entries (isolated 2^21 MSM at c = 20: lo pass 0.269 -> 0.179 ms,
// profiles/r5_lo_scatter_ab.txt). Grouping a region's items on one XCD measured nothing.
template <int LO, int NT = kLoThreads, uint32_t U = kLoU>
__global__ void __launch_bounds__(NT)
msm_lo_scatter_kernel(const typename std::conditional<LO <= 8, uint8_t, uint16_t>::type* __restrict__ lo2,
                      const uint32_t* __restrict__ vals2, const uint32_t* __restrict__ counts, uint32_t ntiles,
                      const uint32_t* __restrict__ segoff, uint32_t* __restrict__ sorted) {
  using Lo = typename std::conditional<LO <= 8, uint8_t, uint16_t>::type;
  constexpr uint32_t NL = 1u << LO;
  constexpr uint32_t kLoThreads = NT, kLoU = U;
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
    for (uint32_t u = 0; u < kLoU; u++) r8[u] = k8[u] < NL ? atomicAdd(&lcnt[k8[u]], 1u) : 0u;
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

// offsets[k] = first position of a key >= k in the sorted key array (k = 0..nkeys)
__global__ void __launch_bounds__(kMsmThreads)
msm_offsets_kernel(const uint32_t* __restrict__ skeys, size_t m, uint32_t nkeys, uint32_t* __restrict__ offsets) {
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
// unconverted (a store per bucket run costs a few instructions; the 4 products of a
// conversion would run for the whole wave whenever any lane ends a run, i.e. on most
// iterations); the window sum reads them in that radix.
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

// kLdsIdx (chunk <= kChunk): the workgroup's kMsmThreads x chunk slice of `sorted` is
// staged into LDS by coalesced loads before the additions. Read from HBM one index per
// addition, each lane's chunk 192 B from its neighbour's, the index lines were evicted
// between uses by the table gathers and fetched again (~1 GB of the 3.3 GB a launch
// moved, profiles/r2_fetch_calibration.txt); a gather-only probe over the same stream
// ran 1.08 ms with HBM indices and 0.65 ms with LDS ones (tools/table_probe.hip).
// 49 KB per workgroup: three workgroups (12 waves, the 3 waves per SIMD the kernel is
// compiled for) fit the CU's 160 KB.
// 3 waves per SIMD (<= 168 VGPRs): at 4 (<= 128) the prefetched next point spilled to
// scratch, 80 B stored and reloaded per entry (WRITE_SIZE 2.5 GB per launch; 2.55 -> 2.29 ms).
// The addition's independent products run in interleaved pairs (mul29x2 / sqr29x2: U2 | S2,
// PP | RR, PPP | Q, ZZ3 | ZZZ3), two v_mad_u64_u32 chains per asm statement (round 3:
// 2.295 -> 2.254 ms isolated, bench +1.3 %).
static constexpr uint32_t kLdsStride = kMsmThreads + 1;  // slot-major rows, +1: conflict-free fill
template <bool kLdsIdx>
__global__ void __launch_bounds__(kMsmThreads) __attribute__((amdgpu_waves_per_eu(3, 8)))
msm_accumulate29_kernel(uint32_t chunk, const G1Affine* __restrict__ bases, const uint32_t* __restrict__ sorted,
                        const uint32_t* __restrict__ offsets, uint32_t nkeys, size_t nthreads,
                        Xyzz29* __restrict__ buckets, Xyzz29* __restrict__ carry_own,
                        Xyzz29* __restrict__ carry_cont) {
  __shared__ uint32_t sidx[kLdsIdx ? kChunk * kLdsStride : 1];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;  // < 2^32 (entries / chunk)
  const uint32_t M = offsets[nkeys];
  if (!chunk) {  // sparse tables: derived from the entry count (<= kChunk)
    chunk = dyn_chunk(M);
    tail_prio();
  }
  if (kLdsIdx) {  // chunk <= kChunk; every thread of the workgroup takes part before any exits
    const uint32_t wg0 = (uint32_t)blockIdx.x * kMsmThreads * chunk;
    if (wg0 >= M) return;  // the whole workgroup is past the stream (the sparse grids' bound)
    // j / chunk by a multiply-high: inv = ceil(2^32 / chunk) is exact for j < 2^32 / chunk^2
    const uint32_t inv = (uint32_t)((0x100000000ull + chunk - 1) / chunk);
    for (uint32_t j = threadIdx.x; j < kMsmThreads * chunk; j += kMsmThreads) {
      const uint32_t thr = __umulhi(j, inv), slot = j - thr * chunk;
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
  bool inf = true;
  // software pipeline: the next entry's table point is loaded before this entry's
  // addition, so the gather's latency hides behind ~8k cycles of arithmetic, and the
  // entry after it is read one step earlier still, so that gather's address is in a
  // register when it is issued (no wait on the index load inside an iteration)
  uint32_t ent = index_at(s);
  G1Affine P = bases[ent & 0x7fffffffu];
  uint32_t ent_n = s + 1 < e ? index_at(s + 1) : 0u;
  for (uint32_t pos = s; pos < e;) {
    G1Affine Pn;
    uint32_t ent_nn = 0;
    if (pos + 1 < e) Pn = bases[ent_n & 0x7fffffffu];
    if (pos + 2 < e) ent_nn = index_at(pos + 2);
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
      } else {
        // madd-2008-s (XYZZ + affine): 8 products + 2 squares, in pairs
        F29 U2, S2, PP, RR;
        mul29x2<Fq29>(x, acc.ZZ, y, acc.ZZZ, U2, S2);
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
          mul29x2<Fq29>(acc.ZZ, PP, acc.ZZZ, PPP, ZZ3, ZZZ3);
          // Y3 = R (Q - X3) + (4p - Y1) PPP, one reduction: (6p 12p + 4p 2p) / 2^261 + p < 2p;
          // Q - X3 + 10p (limbs < 2^30.6) and 4p - Y1 (limbs < 2^30) stay unnormalized
          acc.Y = mul2sum29(R, sub29_nn(Q, X3, Fq29W::K10), neg4p29_nn(acc.Y), PPP);
          acc.ZZ = ZZ3;
          acc.ZZZ = ZZZ3;
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
      // next non-empty bucket: a linear walk (one load per bucket; a chunk crosses at
      // most a few boundaries)
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

// Kernels below keep exactly one inlined EC addition per loop body: an inlined
// formula is ~3.5k instructions, and several copies in one loop thrash the shared
// instruction cache (round 1: 2.7 ms for the three-site form).

// sum of a bucket's carries: the owner chunk's and the continuations c0+1..c1
__device__ __forceinline__ G1xyzz sum_run(const G1xyzz* carry_own, const G1xyzz* carry_cont, uint32_t c0,
                                          uint32_t c1) {
  G1xyzz v = carry_own[c0];
  for (uint32_t u = c0 + 1; u <= c1; u++) v = xyzz_add(v, carry_cont[u]);
  return v;
}

// Buckets whose entries span several accumulation chunks (generic schedule): owner chunk's
// carry plus the continuation carries of the chunks the bucket spills into (thread per
// bucket), into `buckets` (single-chunk ones are already there); runs of more than `span`
// carries go to the large list.
__global__ void __launch_bounds__(kMsmThreads)
msm_bucket_finalize_kernel(uint32_t chunk, const uint32_t* __restrict__ offsets, uint32_t nkeys, uint32_t span,
                           const G1xyzz* __restrict__ carry_own, const G1xyzz* __restrict__ carry_cont,
                           G1xyzz* __restrict__ buckets, uint32_t* __restrict__ large) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nkeys) return;
  const uint32_t s = offsets[k], e = offsets[k + 1];
  if (e == s) return;
  const uint32_t c0 = s / chunk, c1 = (e - 1) / chunk;
  if (c0 == c1) return;  // stored by the accumulation
  if (c1 - c0 > span) {  // long run (skewed digits)
    large[1 + atomicAdd(&large[0], 1u)] = (uint32_t)k;
    return;
  }
  buckets[k] = sum_run(carry_own, carry_cont, c0, c1);
}

// The fixed-base finalize (radix 2^29). Thread per bucket, as above, but a bucket's carries
// past the first addition are not walked by its own lane: at c = 20 (~52 entries per bucket,
// 48-entry chunks) ~92 % of the multi-chunk buckets need exactly one addition, and a wave
// whose longest lane needed 2-6 ran that many rounds of additions for all 64 lanes. Every
// lane does its first addition in one round; the workgroup's buckets with more park their
// partial sum in place (out29) and their carry range in LDS (12 B each: the kernel keeps
// the accumulation's LDS free), and the first waves finish them after a barrier (usually
// one wave, one more round). Isolated 2^21 MSM: 0.149 -> 0.12 ms, VALU -34 %.
__global__ void __launch_bounds__(kMsmThreads)
msm_finalize29_kernel(uint32_t chunk, const uint32_t* __restrict__ offsets, uint32_t nkeys, uint32_t span,
                      const Xyzz29* __restrict__ carry_own, const Xyzz29* __restrict__ carry_cont,
                      uint32_t* __restrict__ large, Xyzz29* __restrict__ out29) {
  tail_prio();
  __shared__ uint32_t pk[kMsmThreads], pu[kMsmThreads], pe[kMsmThreads];
  __shared__ uint32_t cnt;
  if (threadIdx.x == 0) cnt = 0;
  if (!chunk) chunk = dyn_chunk(offsets[nkeys]);  // sparse tables
  __syncthreads();
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t c0 = 0, c1 = 0;
  bool mine = false;
  if (k < nkeys) {
    const uint32_t s = offsets[k], e = offsets[k + 1];
    if (e != s) {
      c0 = s / chunk;
      c1 = (e - 1) / chunk;
      if (c1 - c0 > span)  // long run (skewed digits): msm_large_*
        large[1 + atomicAdd(&large[0], 1u)] = (uint32_t)k;
      else
        mine = c1 > c0;  // single-chunk buckets were stored by the accumulation
    }
  }
  if (mine) {
    out29[k] = add29(carry_own[c0], carry_cont[c0 + 1]);
    if (c1 > c0 + 1) {
      const uint32_t i = atomicAdd(&cnt, 1u);
      pk[i] = (uint32_t)k;
      pu[i] = c0 + 2;
      pe[i] = c1;
    }
  }
  __syncthreads();  // (workgroup-scope fence: the parked sums are visible to the finishing lanes)
  if (threadIdx.x < cnt) {
    const uint32_t kk = pk[threadIdx.x], u1 = pe[threadIdx.x];
    Xyzz29 v = out29[kk];
    for (uint32_t u = pu[threadIdx.x]; u <= u1; u++) v = add29(v, carry_cont[u]);
    out29[kk] = v;
  }
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

// Buckets listed by the finalize kernel (more than kSeqSpan carries, e.g. many equal
// digits): one workgroup per bucket, kSumThreads-way partial sums + LDS tree.
__global__ void __launch_bounds__(kSumThreads)
msm_bucket_large_kernel(uint32_t chunk, const uint32_t* __restrict__ offsets, const uint32_t* __restrict__ large,
                        const G1xyzz* __restrict__ carry_own, const G1xyzz* __restrict__ carry_cont,
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
      rhs = u ? carry_cont[c0 + u] : carry_own[c0];
      return true;
    });
    if (threadIdx.x == 0) buckets[k] = r;
    __syncthreads();
  }
}

// Fixed-base schedule, long carry runs (skewed digits: the Lagrange-basis commitments'
// |digit| = 1 bucket holds ~40 % of their entries, tens of thousands of carries; "equal"
// scalars in the tests): the runs are cut into pieces of kPieceCarries, each summed by one
// workgroup in an LDS tree of ceil(log2(carries)) levels, then one workgroup per bucket adds
// its pieces by another tree (round 6; until round 5 1024-carry pieces, four sequential
// additions per thread before an 8-level tree, and a 64-lane tree over the pieces: 20+
// dependent additions whatever the run's length, on 128 workgroups that walked the pieces
// one after another).
static constexpr uint32_t kPieceCarries = (uint32_t)kSumThreads;

__device__ __forceinline__ uint32_t carry_span(uint32_t chunk, const uint32_t* offsets, uint32_t k, uint32_t* c0) {
  *c0 = offsets[k] / chunk;
  return (offsets[k + 1] - 1) / chunk - *c0 + 1;
}

// off[i] = pieces of the listed buckets before i, off[count] = all (one workgroup).
// chunk 0: the sparse schedule's device-derived chunk (dyn_chunk)
__global__ void __launch_bounds__(1024)
msm_large_scan_kernel(uint32_t chunk, const uint32_t* __restrict__ offsets, uint32_t nkeys,
                      const uint32_t* __restrict__ large, uint32_t* __restrict__ off) {
  tail_prio();
  __shared__ uint32_t sh[1024];
  const uint32_t count = large[0];
  const uint32_t ch = chunk ? chunk : dyn_chunk(offsets[nkeys]);
  const uint32_t tid = threadIdx.x;
  const uint32_t per = (count + 1023u) / 1024u;
  const uint32_t i0 = tid * per < count ? tid * per : count;
  const uint32_t i1 = i0 + per < count ? i0 + per : count;
  auto pieces = [&](uint32_t i) {
    uint32_t c0;
    return (carry_span(ch, offsets, large[1 + i], &c0) + kPieceCarries - 1) / kPieceCarries;
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

// Sum of v over the workgroup's first `cnt` threads (cnt <= kSumThreads, uniform; threads >=
// cnt pass anything) by a tree of ceil(log2(cnt)) levels, the first level straight from the
// registers: thread u adds u + h's value (h = the half, rounded up to a power of two) and the
// tree continues in LDS. Result in thread 0. One addition site.
__device__ __forceinline__ Xyzz29 tree_sum29(Xyzz29 v, uint32_t cnt, Xyzz29* sh) {
  const uint32_t u = threadIdx.x;
  uint32_t h = 1;
  while (h < cnt) h <<= 1;
  h >>= 1;  // cnt <= 1: no level
  if (h) {
    if (u >= h && u < cnt) sh[u] = v;
    __syncthreads();
  }
  // level h reads [h, 2h) and then [h / 2, h) is written for the next level: disjoint, so
  // one barrier per level
  for (; h; h >>= 1) {
    if (u < h && u + h < cnt) v = add29(v, sh[u + h]);
    cnt = h;
    if (h > 1) {
      if (u >= (h >> 1) && u < h) sh[u] = v;
      __syncthreads();
    }
  }
  return v;
}

__global__ void __launch_bounds__(kSumThreads)
msm_large_piece29_kernel(uint32_t chunk, const uint32_t* __restrict__ offsets, uint32_t nkeys,
                         const uint32_t* __restrict__ large, const uint32_t* __restrict__ off,
                         const Xyzz29* __restrict__ carry_own, const Xyzz29* __restrict__ carry_cont,
                         Xyzz29* __restrict__ part) {
  tail_prio();
  __shared__ Xyzz29 sh[kSumThreads];
  const uint32_t count = large[0];
  const uint32_t total = off[count];
  const uint32_t ch = chunk ? chunk : dyn_chunk(offsets[nkeys]);
  for (uint32_t item = blockIdx.x; item < total; item += gridDim.x) {
    uint32_t lo = 0, hi = count;  // largest i with off[i] <= item
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (off[mid] <= item) lo = mid; else hi = mid;
    }
    uint32_t c0;
    const uint32_t span = carry_span(ch, offsets, large[1 + lo], &c0);
    const uint32_t first = (item - off[lo]) * kPieceCarries;
    const uint32_t n = span - first < kPieceCarries ? span - first : kPieceCarries;
    const uint32_t u = first + threadIdx.x;
    Xyzz29 v;
    if (threadIdx.x < n) v = u ? carry_cont[c0 + u] : carry_own[c0];
    v = tree_sum29(v, n, sh);
    if (threadIdx.x == 0) part[item] = v;
    __syncthreads();  // sh is reused by the next item
  }
}

// a listed bucket's pieces: one workgroup of NT threads per bucket, a sequential add per
// thread while there are more than NT pieces, then the tree. The dense tables' launch keeps
// one-wave workgroups (64 threads, as until round 5): it finds nothing to do for random
// scalars, and a 4-wave workgroup of 213 VGPRs waited longer for a free SIMD under the
// other lanes' accumulations; the sparse tables' bucket 0 holds hundreds of pieces (256).
template <int NT>
__global__ void __launch_bounds__(NT)
msm_large_final29_kernel(const uint32_t* __restrict__ large, const uint32_t* __restrict__ off,
                         const Xyzz29* __restrict__ part, Xyzz29* __restrict__ out29) {
  tail_prio();
  __shared__ Xyzz29 sh[NT];
  const uint32_t count = large[0];
  for (uint32_t i = blockIdx.x; i < count; i += gridDim.x) {
    const uint32_t p0 = off[i], np = off[i + 1] - p0;
    if (np == 1) {
      if (threadIdx.x == 0) out29[large[1 + i]] = part[p0];
      continue;
    }
    Xyzz29 v;
    if (threadIdx.x < np) v = part[p0 + threadIdx.x];
    for (uint32_t q = threadIdx.x + NT; q < np; q += NT) v = add29(v, part[p0 + q]);
    v = tree_sum29(v, np < NT ? np : NT, sh);
    if (threadIdx.x == 0) out29[large[1 + i]] = v;
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

// ---- fixed-base window sum: the two-dimensional bucket reduction ----------------------
// nb = 2^lb buckets, bucket k of weight k + 1. With k = h 2^a + l (a = ceil(lb / 2) low
// bits l, hb = lb - a high bits h):
//   W = sum_k (k + 1) B_k = 2^a sum_h h Row_h + sum_l (l + 1) Col_l,
//   Row_h = sum_l B_{h 2^a + l} (2^a consecutive buckets), Col_l = sum_h B_{h 2^a + l},
// so every bucket is added twice, into plain sums, and the only weighted sums left are
// over the 2^hb rows and 2^a columns, done as bit slots (sum_b 2^b S_b with S_b the sum of
// the lines whose index has bit b set) over <= 2^10 terms each. The running-sum reduction
// it replaces (round 3: a thread per 4-bucket segment, 2 L dependent additions, then bit
// slots over the 2^(lb-2) segments) did ~2.4 additions per bucket at c = 20 in chains of
// ~25; here every level is a plain sum with at most 4 + 7 + 12 dependent additions:
//   msm_tile29_kernel   a 16 x 16 tile of buckets per workgroup: the tile's 16 row
//                       partials (over its 16 columns) and 16 column partials (over its 16
//                       rows) by one 4-level LDS tree for both (256 + 128 + 64 + 32
//                       additions: 4 + 2 + 1 + 1 wave-additions per tile)
//   msm_lines29_kernel  kLineThreads threads per line: Row_h over its 2^a / 16 row
//                       partials, Col_l over its 2^hb / 16 column partials
//   msm_slots29_kernel  a workgroup per slot: hb row bits, a column bits, and the plain
//                       column sum (the "+ 1" of the weights); msm_finish combines the
//                       slots on the host: W = 2^a sum_b 2^b R_b + sum_b 2^b C_b + C
static constexpr int kTileSide = 16;
static constexpr int kLineThreads = 8;  // a power of two dividing 64

// sets (BinSets): set s = blockIdx.y, its buckets from s 2^(a + hb), its partials from s times
// one set's row / column partial counts
__global__ void __launch_bounds__(256)
msm_tile29_kernel(const Xyzz29* __restrict__ buckets, const uint32_t* __restrict__ offsets, int a, int ltiles,
                  int htiles, Xyzz29* __restrict__ rowp, Xyzz29* __restrict__ colp) {
  tail_prio();
  // [0, 256): the tile's buckets, then the row tree in place; [256, 384): the column tree
  __shared__ Xyzz29 sh[384];
  const int tid = threadIdx.x;
  const int ht = blockIdx.x / ltiles, lt = blockIdx.x - ht * ltiles;
  {
    const size_t per = (size_t)ltiles * htiles * kTileSide;  // row (= column) partials of one set
    buckets += (size_t)blockIdx.y * ltiles * htiles * kTileSide * kTileSide;
    offsets += (size_t)blockIdx.y * ltiles * htiles * kTileSide * kTileSide;
    rowp += blockIdx.y * per;
    colp += blockIdx.y * per;
  }
  {
    const int i = tid >> 4, j = tid & 15;
    const uint32_t k = ((uint32_t)(ht * kTileSide + i) << a) + (uint32_t)(lt * kTileSide + j);
    sh[tid] = offsets[k + 1] != offsets[k] ? buckets[k] : pinf<Xyzz29>();
  }
  __syncthreads();
  // level s (m = 8 >> s): 16 m row additions (row i: j += j + m, j < m) on threads
  // [0, 16 m), 16 m column additions (column j: i += i + m, i < m) on [16 m, 32 m); the
  // first column level reads the buckets, later ones the column tree
#pragma unroll 1
  for (int s = 0; s < 4; s++) {
    const int m = 8 >> s;
    const bool act = tid < 32 * m;
    int l = 0, r = 0, d = 0;
    if (tid < 16 * m) {
      const int i = tid / m, j = tid - i * m;
      l = d = i * 16 + j;
      r = l + m;
    } else if (act) {
      const int u = tid - 16 * m, i = u >> 4, j = u & 15;
      const int base = s ? 256 : 0;
      l = base + i * 16 + j;
      r = base + (i + m) * 16 + j;
      d = 256 + i * 16 + j;
    }
    Xyzz29 x, y;
    if (act) {
      x = sh[l];
      y = sh[r];
    }
    __syncthreads();
    if (act) sh[d] = add29(x, y);
    __syncthreads();
  }
  if (tid < kTileSide)
    rowp[(size_t)(ht * kTileSide + tid) * ltiles + lt] = sh[tid * 16];
  else if (tid < 2 * kTileSide)
    colp[(size_t)(lt * kTileSide + tid - kTileSide) * htiles + ht] = sh[256 + tid - kTileSide];
}

// The same first level for the wide windows (c >= 19, 2^18+ buckets; round 5): strips
// instead of LDS tiles. Row partials: thread (h, j), j < RJ = 2^a / kStrip, adds the buckets
// (h, j + RJ t), t < kStrip, so consecutive threads read consecutive buckets; column partials:
// thread (i, l), i < CI = 2^hb / kStrip, adds (i + CI t, l), consecutive threads consecutive
// l. Every bucket is read and added twice, as in the tiles, with every lane busy and no LDS or
// barrier: at 2^19 buckets the tile kernel's 55 KB of LDS per workgroup kept the bucket
// accumulation's third workgroup off a CU whenever the two shared one (5 proof lanes).
// rowp[h RJ + j], colp[l CI + i]: the layout msm_lines29_kernel reads (RJ, CI partials a line).
static constexpr int kStrip = 16;
static constexpr int kStripMinC = 19;  // the tiles stay for c <= 18 (2^16 buckets: 0.046 ms, shorter chains)
__global__ void __launch_bounds__(256)
msm_strips29_kernel(const Xyzz29* __restrict__ buckets, const uint32_t* __restrict__ offsets, int a, int hb,
                    Xyzz29* __restrict__ rowp, Xyzz29* __restrict__ colp) {
  tail_prio();
  const int RJ = (1 << a) / kStrip, CI = (1 << hb) / kStrip;
  const size_t nrow = (size_t)RJ << hb, ncol = (size_t)CI << a;
  const size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= nrow + ncol) return;
  uint32_t k, step;
  size_t dst;
  Xyzz29* out;
  if (g < nrow) {
    const uint32_t h = (uint32_t)(g / RJ), j = (uint32_t)(g % RJ);
    k = (h << a) + j;
    step = (uint32_t)RJ;
    dst = g;
    out = rowp;
  } else {
    const size_t u = g - nrow;
    const uint32_t i = (uint32_t)(u >> a), l = (uint32_t)(u & ((1u << a) - 1));
    k = (i << a) + l;
    step = (uint32_t)CI << a;
    dst = (size_t)l * CI + i;
    out = colp;
  }
  Xyzz29 acc = pinf<Xyzz29>();
#pragma unroll 1
  for (int t = 0; t < kStrip; t++, k += step) {
    const Xyzz29 y = offsets[k + 1] != offsets[k] ? buckets[k] : pinf<Xyzz29>();
    acc = add29(acc, y);
  }
  out[dst] = acc;
}

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

// lines [0, nrows) are rows (ltiles partials each), [nrows, nrows + ncols) columns (htiles
// partials each); kLineThreads consecutive lanes per line: a strided sequential sum, then a
// butterfly over the group (one addition site; the shuffles run on every step's wave, the
// sequential part's bound is wave-uniform)
__global__ void __launch_bounds__(256)
msm_lines29_kernel(const Xyzz29* __restrict__ rowp, int ltiles, const Xyzz29* __restrict__ colp, int htiles,
                   int nrows, int ncols, Xyzz29* __restrict__ lines) {
  tail_prio();
  // sets: set s = blockIdx.y (one set's partials: nrows ltiles = ncols htiles; lines nrows + ncols)
  rowp += (size_t)blockIdx.y * nrows * ltiles;
  colp += (size_t)blockIdx.y * ncols * htiles;
  lines += (size_t)blockIdx.y * (nrows + ncols);
  constexpr int LG = kLineThreads == 8 ? 3 : kLineThreads == 4 ? 2 : kLineThreads == 16 ? 4 : 1;
  static_assert((1 << LG) == kLineThreads, "kLineThreads: 2, 4, 8 or 16");
  const int g = (int)((blockIdx.x * 256 + threadIdx.x) / kLineThreads);
  const int r = (int)(threadIdx.x & (kLineThreads - 1));
  const bool live = g < nrows + ncols;
  const bool row = g < nrows;
  const Xyzz29* src = row ? rowp + (size_t)g * ltiles : colp + (size_t)(g - nrows) * htiles;
  const int cnt = live ? (row ? ltiles : htiles) : 0;
  const int maxcnt = ltiles > htiles ? ltiles : htiles;
  const int nseq = (maxcnt + kLineThreads - 1) / kLineThreads - 1;  // after the first term
  Xyzz29 acc = r < cnt ? src[r] : pinf<Xyzz29>();
#pragma unroll 1
  for (int step = 0; step < nseq + LG; step++) {
    Xyzz29 y;
    if (step < nseq) {
      const int q = r + (step + 1) * kLineThreads;
      y = q < cnt ? src[q] : pinf<Xyzz29>();
    } else {
      y = shfl_xor29(acc, 1 << (step - nseq));
    }
    acc = add29(acc, y);
  }
  if (live && r == 0) lines[g] = acc;
}

// slot s < hb: the rows with bit s set; hb <= s < hb + a: the columns with bit s - hb set;
// s = hb + a: every column. Converted to the 8x32 layout and written straight into the
// scratch's pinned host_win (round 6: the copy after the kernel was one more blit dispatch per
// MSM, queued behind the other lanes' kernels), with the bucketed entry count when total_out
// is set (kernel statistics).
__global__ void __launch_bounds__(kSumThreads)
msm_slots29_kernel(const Xyzz29* __restrict__ lines, int hb, int a, G1xyzz* __restrict__ out,
                   const uint32_t* __restrict__ entries, uint32_t* __restrict__ total_out) {
  tail_prio();
  // sets: set = blockIdx.y (its lines from set (2^hb + 2^a), its slots from set (hb + a + 1))
  lines += (size_t)blockIdx.y * (((size_t)1 << hb) + ((size_t)1 << a));
  out += (size_t)blockIdx.y * (hb + a + 1);
  __shared__ Xyzz29 sh[kSumThreads];
  const int s = blockIdx.x;
  const bool rows = s < hb;
  const bool plain = s == hb + a;
  const int b = rows ? s : s - hb;
  const int count = plain ? 1 << a : (rows ? 1 << (hb - 1) : 1 << (a - 1));
  const Xyzz29* src = rows ? lines : lines + ((size_t)1 << hb);
  const int per = (count + kSumThreads - 1) / kSumThreads;
  const Xyzz29 r = block_sum<kSumThreads>(per, sh, [&](int step, Xyzz29& rhs) {
    const int q = step * kSumThreads + (int)threadIdx.x;
    if (q >= count) return false;
    rhs = src[plain ? q : (((q >> b) << (b + 1)) | (1 << b) | (q & ((1 << b) - 1)))];
    return true;
  });
  if (threadIdx.x == 0) {  // pinned host memory (common.h host_put)
    host_put(out + s, load_point(r));
    if (s == 0 && blockIdx.y == 0 && total_out) host_put(total_out, *entries);
    host_put_done();
  }
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
  q.alloc((size_t)nw * stride);
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

// NZCB_MARK_LAUNCHES=1: a roctx mark after every launch of the fixed-base schedule, so that a
// rocprofv3 --marker-trace shows the host time each launch takes inside a proof (round 6:
// round 1's commitments were enqueued ~0.5-1 ms apart)
static void lmark(const char* what) {
  static const bool on = std::getenv("NZCB_MARK_LAUNCHES") != nullptr;
  if (on) roctxMarkA(what);
}

// work items of the bucket_lo steps: at most one partial segment per region + entries / kLoSeg
static size_t lo_items_bound(size_t entries) { return 256 + entries / kLoSeg + 1; }

struct MsmPlan {
  int c, nw, nsets, seglen, nseg, nbits, nslots, nparts;
  int lb, a, hb, ltiles, htiles;  // fixed base: the two-dimensional window sum
  int msets;                      // fixed base: MSMs sharing the schedule (BinSets)
  uint32_t nb, nkeys;
  size_t entries;
};

static MsmPlan make_plan(size_t n, const MsmBaseTable* t, int msets = 1) {
  MsmPlan p;
  p.c = t ? t->c : msm_window_bits(n);
  p.nw = num_windows(p.c);
  p.nsets = t ? 1 : p.nw;
  p.msets = t ? msets : 1;
  p.nb = 1u << (p.c - 1);
  p.nkeys = p.nb * (uint32_t)p.nsets * (uint32_t)p.msets;
  p.seglen = (int)(p.nb < (uint32_t)kSegLen ? p.nb : kSegLen);
  p.nseg = (int)(p.nb / p.seglen);
  p.nbits = 0;
  while ((1 << p.nbits) < p.nseg) p.nbits++;
  p.nslots = p.nbits + 1;
  p.nparts = (p.nseg + kSumThreads * kSumPer - 1) / (kSumThreads * kSumPer);
  p.lb = p.c - 1;
  p.a = (p.lb + 1) / 2;
  p.hb = p.lb - p.a;
  p.ltiles = (1 << p.a) / kTileSide;
  p.htiles = (1 << p.hb) / kTileSide;
  p.entries = n * (size_t)p.nw * (size_t)p.msets;
  return p;
}

void MsmScratch::init(size_t maxp, bool fixed_base, int lagrange_sets, bool generic) {
  if (lagrange_sets < 1 || lagrange_sets > kMaxSets) throw Error(NZCB_ERR_ARG, "msm scratch: 1..3 Lagrange sets");
  if (!fixed_base) generic = true;
  max_points = maxp;
  max_lsets = lagrange_sets;
  size_t max_entries = 0, max_keys = 0, max_seg = 0, max_slots = 0, max_parts = 0, max_tiles = 0, max_lines = 0;
  auto fit = [&](const MsmPlan& p) {
    max_entries = std::max(max_entries, p.entries);
    max_keys = std::max(max_keys, (size_t)p.nkeys);
    if (p.nsets == 1) {  // fixed base
      max_slots = std::max(max_slots, (size_t)(p.lb + 1) * p.msets);
      max_tiles = std::max(max_tiles, (size_t)p.nb / kTileSide * p.msets);
      max_lines = std::max(max_lines, (((size_t)1 << p.hb) + ((size_t)1 << p.a)) * p.msets);
    } else {
      max_seg = std::max(max_seg, (size_t)p.nseg * p.nsets);
      max_slots = std::max(max_slots, (size_t)p.nslots * p.nsets);
      max_parts = std::max(max_parts, (size_t)p.nslots * p.nsets * p.nparts);
    }
  };
  for (size_t n = 1;; n <<= 1) {
    size_t m = n < maxp ? n : maxp;
    fit(make_plan(m, nullptr));
    if (m == maxp) break;
  }
  MsmPlan fp{};
  if (fixed_base) {  // the PTau tables' window and the Lagrange table's
    MsmBaseTable t;
    t.c = fixed_base_window();
    fp = make_plan(maxp, &t);
    fit(fp);
    t.c = lagrange_window();
    const MsmPlan lp = make_plan(maxp, &t, lagrange_sets);
    fit(lp);
    if (lp.entries > fp.entries) fp = lp;
  }
  // generic = false (the prover's and the serving ranks' scratches, which only run tables):
  // none of the generic schedule's sort, 8x32 bucket and segment arrays
  const size_t ge = generic ? max_entries : 1;
  offsets.alloc(max_keys + 1);
  sorted.alloc(max_entries);
  keys_in.alloc(ge);
  keys_out.alloc(max_entries);  // the fixed-base bucketing's low key parts
  vals_in.alloc(ge);
  sort_tmp_bytes = 0;
  if (generic) {
    radix_sort(nullptr, sort_tmp_bytes, keys_in.p, keys_out.p, vals_in.p, sorted.p, max_entries, 21, nullptr);
  }
  sort_tmp.alloc(sort_tmp_bytes + 16);
  // accumulation threads: chunk_for's grid, or the sparse schedule's (dyn_threads_bound)
  const size_t nthreads = std::max((max_entries + kChunk - 1) / kChunk, dyn_threads_bound(max_entries)) + 1;
  buckets.alloc(generic ? max_keys : 1);
  carry_own.alloc(generic ? nthreads : 1);
  carry_cont.alloc(generic ? nthreads : 1);
  large.alloc(max_keys + 1);
  if (fixed_base) {
    buckets29.alloc(max_keys);
    large_off.alloc(max_keys + 2);
    // pieces: sum over listed buckets of ceil(span / kPieceCarries) <= chunks / kPieceCarries + buckets
    large_part.alloc(nthreads / kPieceCarries + max_keys + 1);
    carry_own29.alloc(nthreads);
    carry_cont29.alloc(nthreads);
    rowp29.alloc(max_tiles);
    colp29.alloc(max_tiles);
    lines29.alloc(max_lines);
    bin_counts.alloc((size_t)256 * ((maxp + kTileScalars - 1) / kTileScalars) * lagrange_sets + 256);  // + row totals
    vals_mid.alloc(max_entries);
    lo_seg.alloc(lo_items_bound(max_entries) * ((size_t)1 << BinKeys<19>::LO));  // the widest low index
  }
  seg_tot.alloc(max_seg && generic ? max_seg : 1);
  seg_run.alloc(max_seg && generic ? max_seg : 1);
  parts.alloc(max_parts && generic ? max_parts : 1);
  win.alloc(max_slots);
  host_win_cap = max_slots;
  // coherent: the fixed-base window sums are written here by msm_slots29_kernel
  NZ_HIP(hipHostMalloc((void**)&host_win, (max_slots + 1) * sizeof(G1xyzz), hipHostMallocCoherent));
  host_total = (uint32_t*)(host_win + max_slots);  // one more slot: the profiled entry count
}

MsmScratch::~MsmScratch() {
  if (host_win) (void)hipHostFree(host_win);
  if (done) (void)hipEventDestroy(done);
  for (auto& e : ev)
    if (e) (void)hipEventDestroy(e);
}

static void keys_dispatch(int c, const Fr* scalars, size_t n, int mont, MsmScratch& sc, hipStream_t st) {
  auto launch = [&](auto cc) {
    constexpr int C = decltype(cc)::value;
    hipLaunchKernelGGL(msm_keys_kernel<C>, dim3(grid_for(n, kMsmThreads, 1u << 30)), dim3(kMsmThreads), 0, st,
                       scalars, n, mont, sc.keys_in.p, sc.vals_in.p);
  };
  switch (c) {
#define NZ_CASE(K) case K: launch(std::integral_constant<int, K>()); break;
    NZ_CASE(4) NZ_CASE(5) NZ_CASE(6) NZ_CASE(7) NZ_CASE(8) NZ_CASE(9) NZ_CASE(10) NZ_CASE(11) NZ_CASE(12)
    NZ_CASE(13) NZ_CASE(14) NZ_CASE(15) NZ_CASE(16)
#undef NZ_CASE
    default: throw Error(NZCB_ERR_INTERNAL, "bad msm window");
  }
  NZ_HIP(hipGetLastError());
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

// fixed base: bucketing (msm_bin_* / msm_lo_*) into sc.offsets / sc.sorted
template <class Mark>
static void fixed_bucketing(MsmScratch& sc, const MsmPlan& p, const BinSets& sets, size_t n, int mdig,
                            const MsmBaseTable* table, hipStream_t st, const Mark& mark) {
  const uint32_t tps = (uint32_t)((n + kTileScalars - 1) / kTileScalars);
  const uint32_t ntiles = tps * (uint32_t)p.msets;
  BinSets bs = sets;
  bs.tps = tps;
  bs.nb = p.nb;
  uint32_t* tail = sc.bin_counts.p + (size_t)256 * ntiles;
  auto run_bins = [&](auto cc, auto kb) {
    constexpr int C = decltype(cc)::value;
    constexpr int KB = decltype(kb)::value;  // key bits: c - 1, + 2 for up to 3 sets
    using Lo = typename BinKeys<KB>::Lo;
    constexpr int LO = BinKeys<KB>::LO;
    Lo* lo2 = (Lo*)sc.keys_out.p;
    hipLaunchKernelGGL((msm_bin_hist_kernel<C, KB>), dim3(ntiles), dim3(kBinThreads), 0, st, bs, n, mdig,
                       sc.bin_counts.p, ntiles);
    NZ_HIP(hipGetLastError());
    lmark("mark: L hist");
    mark(1);
    hipLaunchKernelGGL(msm_bin_rowscan_kernel, dim3(256), dim3(256), 0, st, sc.bin_counts.p, ntiles, tail);
    lmark("mark: L rowscan");
    hipLaunchKernelGGL((msm_bin_scatter_kernel<C, KB>), dim3(ntiles), dim3(kBinThreads), 0, st, bs, n, mdig,
                       table->stride, sc.bin_counts.p, ntiles, lo2, sc.vals_mid.p);
    NZ_HIP(hipGetLastError());
    lmark("mark: L scatter");
    mark(2);
    const dim3 igrid((unsigned)lo_items_bound(p.entries));
    hipLaunchKernelGGL(msm_lo_count_kernel<LO>, igrid, dim3(kLoThreads), 0, st, (const Lo*)lo2, sc.bin_counts.p,
                       ntiles, sc.lo_seg.p);
    NZ_HIP(hipGetLastError());
    lmark("mark: L lo_count");
    hipLaunchKernelGGL(msm_lo_scan_kernel<LO>, dim3(256), dim3(kLoThreads), 0, st, sc.bin_counts.p, ntiles,
                       sc.lo_seg.p, p.nkeys, sc.offsets.p, sc.large.p);
    NZ_HIP(hipGetLastError());
    lmark("mark: L lo_scan");
    constexpr int sNT = LO > 8 ? 1024 : kLoThreads;
    constexpr uint32_t sU = LO > 8 ? 16 : kLoU;
    hipLaunchKernelGGL((msm_lo_scatter_kernel<LO, sNT, sU>), igrid, dim3(sNT), 0, st, (const Lo*)lo2, sc.vals_mid.p,
                       sc.bin_counts.p, ntiles, (const uint32_t*)sc.lo_seg.p, sc.sorted.p);
    NZ_HIP(hipGetLastError());
    lmark("mark: L lo_scatter");
  };
  using std::integral_constant;
  if (p.msets > 1) {  // several MSMs: 2 more key bits (up to 4 sets; Lagrange window only)
    if (p.c != 17) throw Error(NZCB_ERR_INTERNAL, "msm sets: the Lagrange window (17) only");
    run_bins(integral_constant<int, 17>(), integral_constant<int, 18>());
    return;
  }
  switch (p.c) {
    case 16: run_bins(integral_constant<int, 16>(), integral_constant<int, 15>()); break;
    case 17: run_bins(integral_constant<int, 17>(), integral_constant<int, 16>()); break;
    case 18: run_bins(integral_constant<int, 18>(), integral_constant<int, 17>()); break;
    case 19: run_bins(integral_constant<int, 19>(), integral_constant<int, 18>()); break;
    case 20: run_bins(integral_constant<int, 20>(), integral_constant<int, 19>()); break;
    default: throw Error(NZCB_ERR_INTERNAL, "bad fixed-base msm window");
  }
}

static void msm_enqueue_impl(MsmScratch& sc, const G1Affine* bases, const Fr* const* scalars, int msets, size_t n,
                             bool mont, hipStream_t st, const MsmBaseTable* table) {
  const auto t_enq = std::chrono::steady_clock::now();
  struct EnqueueClock {  // host time of the enqueue, for the phase timing (nzcb_engine_time_msm2)
    MsmScratch& sc;
    std::chrono::steady_clock::time_point t0;
    ~EnqueueClock() {
      if (sc.prof && sc.prof_phases)
        sc.enqueue_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
  } enqueue_clock{sc, t_enq};
  sc.cur_n = n;
  if (n == 0) return;
  if (!sc.done) NZ_HIP(hipEventCreateWithFlags(&sc.done, hipEventDisableTiming));
  if (n > sc.max_points) throw Error(NZCB_ERR_ARG, "msm larger than scratch");
  if (table && n > table->n) throw Error(NZCB_ERR_ARG, "msm larger than its base table");
  if (table && table->mont_folded && !mont) throw Error(NZCB_ERR_ARG, "2^-256-folded table needs Montgomery scalars");
  if (table && (!sc.buckets29.p || !sc.bin_counts.p))
    throw Error(NZCB_ERR_ARG, "msm scratch was not sized for the fixed-base schedule");
  // a folded table takes the Montgomery form's integer as the scalar (msm_table_kernel)
  const int mdig = (mont && !(table && table->mont_folded)) ? 1 : 0;
  if (msets < 1 || msets > kMaxSets || (msets > 1 && (!table || msets > sc.max_lsets)))
    throw Error(NZCB_ERR_ARG, "msm sets: 1..3 over a table, within the scratch's sizing");
  const MsmPlan p = make_plan(n, table, msets);
#ifdef NZCB_MSM_STATS
  if (table && !table->mont_folded) {  // scalar census (diagnostics build): nonzero c-bit digits of
    // s and of min(s, r - s), the form a per-scalar sign flip would bucket
    NZ_HIP(hipStreamSynchronize(st));
    for (int k = 0; k < msets; k++) {
      std::vector<Fr> h(n);
      NZ_HIP(hipMemcpy(h.data(), scalars[k], n * sizeof(Fr), hipMemcpyDeviceToHost));
      size_t e_pos = 0, e_min = 0, nneg = 0, zero = 0, hist[17] = {0};
      for (size_t i = 0; i < n; i++) {
        Fr v = mdig ? from_mont(h[i]) : h[i];
        if (v.is_zero()) { zero++; continue; }
        const Fr w = neg(v);  // r - v
        auto digits = [&](const Fr& x) {
          size_t d = 0;
          for_each_digit_host(x, p.c, [&](int, uint32_t, uint32_t) { d++; });
          return d;
        };
        const size_t dp = digits(v), dn = digits(w);
        e_pos += dp;
        e_min += dp <= dn ? dp : dn;
        if (dn < dp) nneg++;
        const size_t dm = dp <= dn ? dp : dn;
        hist[dm < 16 ? dm : 16]++;
      }
      fprintf(stderr, "MSMSCALARS set=%d n=%zu c=%d zero=%zu entries=%zu entries_minform=%zu flipped=%zu hist_minform=",
              k, n, p.c, zero, e_pos, e_min, nneg);
      for (int b = 0; b < 17; b++) fprintf(stderr, "%zu%c", hist[b], b == 16 ? '\n' : ',');
    }
  }
#endif
  if (p.entries > sc.sorted.n || p.nkeys + 1 > sc.offsets.n)
    throw Error(NZCB_ERR_ARG, "msm scratch was not sized for this schedule");
  if (table && ((size_t)p.nb / kTileSide * msets > sc.rowp29.n ||
                (((size_t)1 << p.hb) + ((size_t)1 << p.a)) * msets > sc.lines29.n ||
                (size_t)(p.lb + 1) * msets > sc.host_win_cap || (msets > 1 && p.c >= kStripMinC)))
    throw Error(NZCB_ERR_ARG, "msm scratch was not sized for this window");
  sc.cur_c = p.c;
  sc.cur_nsets = p.nsets;
  sc.cur_nbits = p.nbits;
  sc.cur_seglen = p.seglen;
  sc.cur_nkeys = p.nkeys;
  sc.cur_fixed = table != nullptr;
  sc.cur_a = p.a;
  sc.cur_hb = p.hb;
  sc.cur_msets = p.msets;
  const bool phases = sc.prof && sc.prof_phases;
  if (sc.prof && !sc.ev[0])
    for (auto& e : sc.ev) NZ_HIP(hipEventCreate(&e));
  auto mark = [&](int i) {
    if (phases) NZ_HIP(hipEventRecord(sc.ev[i], st));
  };
  mark(0);
  if (table) {
    BinSets bs{};
    for (int k = 0; k < msets; k++) bs.p[k] = scalars[k];
    fixed_bucketing(sc, p, bs, n, mdig | (table->mont_folded ? 0 : kDigMinForm), table, st, mark);
  } else {
    keys_dispatch(p.c, scalars[0], n, mdig, sc, st);
    mark(1);
    size_t tmp = sc.sort_tmp_bytes;
    int end_bit = 1;
    while ((1u << end_bit) <= p.nkeys) end_bit++;
    const auto t_sort = std::chrono::steady_clock::now();
    radix_sort(sc.sort_tmp.p, tmp, sc.keys_in.p, sc.keys_out.p, sc.vals_in.p, sc.sorted.p, p.entries, end_bit, st);
    if (phases)
      sc.sort_host_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_sort).count();
    mark(2);
    hipLaunchKernelGGL(msm_offsets_kernel, dim3(grid_for((size_t)p.nkeys + 1, kMsmThreads, 1u << 30)),
                       dim3(kMsmThreads), 0, st, sc.keys_out.p, p.entries, p.nkeys, sc.offsets.p);
    NZ_HIP(hipGetLastError());
  }
  if (sc.prof) NZ_HIP(hipEventRecord(sc.ev[3], st));
  // sparse tables: chunk 0 = derived on the device from the bucketed entry count (dyn_chunk);
  // the grid covers the most threads any count can ask for
  const bool sparse = table && table->sparse;
  sc.cur_sparse = sparse;
  const uint32_t chunk = sparse ? 0u : chunk_for(p.entries);
  const size_t nthreads = sparse ? dyn_threads_bound(p.entries) : (p.entries + chunk - 1) / chunk;
  const dim3 agrid(grid_for(nthreads, kMsmThreads, 1u << 30));
  const G1Affine* gather = table ? table->q.p : bases;
  if (table) {
    if (chunk == kChunk || sparse)  // sparse: chunk <= kChunk
      hipLaunchKernelGGL(msm_accumulate29_kernel<true>, agrid, dim3(kMsmThreads), 0, st, chunk, gather, sc.sorted.p,
                         sc.offsets.p, p.nkeys, nthreads, sc.buckets29.p, sc.carry_own29.p, sc.carry_cont29.p);
    else
      hipLaunchKernelGGL(msm_accumulate29_kernel<false>, agrid, dim3(kMsmThreads), 0, st, chunk, gather, sc.sorted.p,
                         sc.offsets.p, p.nkeys, nthreads, sc.buckets29.p, sc.carry_own29.p, sc.carry_cont29.p);
  } else {
    hipLaunchKernelGGL(msm_accumulate_kernel, agrid, dim3(kMsmThreads), 0, st, chunk, gather, sc.sorted.p, sc.offsets.p,
                       p.nkeys, nthreads, sc.buckets.p, sc.carry_own.p, sc.carry_cont.p);
  }
  NZ_HIP(hipGetLastError());
  lmark("mark: L accumulate");
  if (sc.prof) NZ_HIP(hipEventRecord(sc.ev[4], st));
  const dim3 fgrid(grid_for(p.nkeys, kMsmThreads, 1u << 30));
  if (table) {  // the large list's count was zeroed by msm_lo_scan_kernel
    hipLaunchKernelGGL(msm_finalize29_kernel, fgrid, dim3(kMsmThreads), 0, st, chunk, sc.offsets.p, p.nkeys,
                       sparse ? kSeqSpanSparse : kSeqSpan29, (const Xyzz29*)sc.carry_own29.p,
                       (const Xyzz29*)sc.carry_cont29.p, sc.large.p, sc.buckets29.p);
    NZ_HIP(hipGetLastError());
    lmark("mark: L finalize");
    hipLaunchKernelGGL(msm_large_scan_kernel, dim3(1), dim3(1024), 0, st, chunk, sc.offsets.p, p.nkeys, sc.large.p,
                       sc.large_off.p);
    NZ_HIP(hipGetLastError());
    lmark("mark: L large_scan");
    hipLaunchKernelGGL(msm_large_piece29_kernel, dim3(sparse ? kSparsePieceBlocks : kLargePieceBlocks),
                       dim3(kSumThreads), 0, st, chunk, sc.offsets.p, p.nkeys, sc.large.p, sc.large_off.p,
                       (const Xyzz29*)sc.carry_own29.p, (const Xyzz29*)sc.carry_cont29.p, sc.large_part.p);
    NZ_HIP(hipGetLastError());
    lmark("mark: L piece");
    if (sparse)
      hipLaunchKernelGGL(msm_large_final29_kernel<kSumThreads>, dim3(kSparseFinalBlocks), dim3(kSumThreads), 0, st,
                         sc.large.p, sc.large_off.p, sc.large_part.p, sc.buckets29.p);
    else
      hipLaunchKernelGGL(msm_large_final29_kernel<64>, dim3(kLargeFinalBlocks), dim3(64), 0, st, sc.large.p,
                         sc.large_off.p, sc.large_part.p, sc.buckets29.p);
    NZ_HIP(hipGetLastError());
    lmark("mark: L final");
    mark(5);
    int lparts = p.ltiles, hparts = p.htiles;  // partials per row / per column
    if (p.c >= kStripMinC) {
      lparts = (1 << p.a) / kStrip;
      hparts = (1 << p.hb) / kStrip;
      const size_t nthr = ((size_t)lparts << p.hb) + ((size_t)hparts << p.a);
      hipLaunchKernelGGL(msm_strips29_kernel, dim3(grid_for(nthr, 256, 1u << 30)), dim3(256), 0, st,
                         (const Xyzz29*)sc.buckets29.p, sc.offsets.p, p.a, p.hb, sc.rowp29.p, sc.colp29.p);
    } else {
      hipLaunchKernelGGL(msm_tile29_kernel, dim3((unsigned)(p.ltiles * p.htiles), (unsigned)p.msets), dim3(256), 0, st,
                         (const Xyzz29*)sc.buckets29.p, sc.offsets.p, p.a, p.ltiles, p.htiles, sc.rowp29.p, sc.colp29.p);
    }
    NZ_HIP(hipGetLastError());
    mark(6);
    const int nrows = 1 << p.hb, ncols = 1 << p.a;
    hipLaunchKernelGGL(msm_lines29_kernel, dim3(grid_for((size_t)(nrows + ncols) * kLineThreads, 256), (unsigned)p.msets),
                       dim3(256), 0,
                       st, (const Xyzz29*)sc.rowp29.p, lparts, (const Xyzz29*)sc.colp29.p, hparts, nrows, ncols,
                       sc.lines29.p);
    NZ_HIP(hipGetLastError());
    lmark("mark: L lines");
    hipLaunchKernelGGL(msm_slots29_kernel, dim3(p.hb + p.a + 1, (unsigned)p.msets), dim3(kSumThreads), 0, st,
                       (const Xyzz29*)sc.lines29.p, p.hb, p.a, sc.host_win, (const uint32_t*)sc.offsets.p + p.nkeys,
                       sc.prof ? sc.host_total : nullptr);
    NZ_HIP(hipGetLastError());
    lmark("mark: L slots");
    mark(7);
    NZ_HIP(hipEventRecord(sc.done, st));
    return;
  }
  NZ_HIP(hipMemsetAsync(sc.large.p, 0, sizeof(uint32_t), st));
  hipLaunchKernelGGL(msm_bucket_finalize_kernel, fgrid, dim3(kMsmThreads), 0, st, chunk, sc.offsets.p, p.nkeys,
                     kSeqSpan, (const G1xyzz*)sc.carry_own.p, (const G1xyzz*)sc.carry_cont.p, sc.buckets.p, sc.large.p);
  NZ_HIP(hipGetLastError());
  hipLaunchKernelGGL(msm_bucket_large_kernel, dim3(kLargeBlocks), dim3(kSumThreads), 0, st, chunk, sc.offsets.p,
                     sc.large.p, (const G1xyzz*)sc.carry_own.p, (const G1xyzz*)sc.carry_cont.p, sc.buckets.p);
  NZ_HIP(hipGetLastError());
  mark(5);
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
  if (sc.prof) NZ_HIP(hipMemcpyAsync(sc.host_total, sc.offsets.p + p.nkeys, 4, hipMemcpyDeviceToHost, st));
  NZ_HIP(hipMemcpyAsync(sc.host_win, sc.win.p, (size_t)p.nsets * p.nslots * sizeof(G1xyzz), hipMemcpyDeviceToHost,
                        st));
  NZ_HIP(hipEventRecord(sc.done, st));
}

void msm_enqueue(MsmScratch& sc, const G1Affine* bases, const Fr* scalars, size_t n, bool mont, hipStream_t st,
                 const MsmBaseTable* table) {
  const Fr* one[1] = {scalars};
  msm_enqueue_impl(sc, bases, one, 1, n, mont, st, table);
}

void msm_enqueue_sets(MsmScratch& sc, const Fr* const* scalars, int sets, size_t n, bool mont, hipStream_t st,
                      const MsmBaseTable* table) {
  if (!table) throw Error(NZCB_ERR_ARG, "msm sets: a table schedule");
  msm_enqueue_impl(sc, nullptr, scalars, sets, n, mont, st, table);
}

// the fixed-base slots of set s combined on the host: W = 2^a sum_b 2^b R_b + sum_b 2^b C_b + C
static G1xyzz fixed_window_result(const G1xyzz* s, int hb, int a) {
  G1xyzz acc = G1xyzz::inf();
  for (int b = hb - 1; b >= 0; b--) acc = xyzz_add(xyzz_dbl(acc), s[b]);
  for (int i = 0; i < a; i++) acc = xyzz_dbl(acc);
  G1xyzz col = G1xyzz::inf();
  for (int b = a - 1; b >= 0; b--) col = xyzz_add(xyzz_dbl(col), s[hb + b]);
  return xyzz_add(xyzz_add(acc, col), s[hb + a]);
}

void msm_finish_sets(MsmScratch& sc, hipStream_t st, G1xyzz* out) {
  const int msets = sc.cur_msets;
  if (sc.cur_n == 0) {
    for (int k = 0; k < msets; k++) out[k] = G1xyzz::inf();
    return;
  }
  out[0] = msm_finish(sc, st);  // waits, timings, set 0
  for (int k = 1; k < msets; k++) out[k] = fixed_window_result(sc.host_win + (size_t)k * (sc.cur_hb + sc.cur_a + 1),
                                                               sc.cur_hb, sc.cur_a);
}

G1xyzz msm_finish(MsmScratch& sc, hipStream_t st) {
  if (sc.cur_n == 0) return G1xyzz::inf();
  // the window sums' copy, not the whole stream: work queued on the stream after the MSM
  // (the prover's A/B/C interpolations follow C's commitment on its stream) runs on
  NZ_HIP(hipEventSynchronize(sc.done));
#ifdef NZCB_MSM_STATS
  if (sc.cur_fixed) {  // scratch diagnostics build: carry spans of the buckets
    std::vector<uint32_t> off(sc.cur_nkeys + 1);
    NZ_HIP(hipMemcpy(off.data(), sc.offsets.p, off.size() * 4, hipMemcpyDeviceToHost));
    uint32_t cnt = 0;
    NZ_HIP(hipMemcpy(&cnt, sc.large.p, 4, hipMemcpyDeviceToHost));
    uint32_t pieces = 0;
    NZ_HIP(hipMemcpy(&pieces, sc.large_off.p + cnt, 4, hipMemcpyDeviceToHost));
    const uint32_t M = off.back();
    const uint32_t chunk = sc.cur_sparse ? dyn_chunk(M) : chunk_for(sc.cur_n * (size_t)num_windows(sc.cur_c));
    size_t h[12] = {0};
    uint32_t mx = 0;
    uint64_t carries_large = 0, carries_mid = 0;
    for (uint32_t k = 0; k < sc.cur_nkeys; k++) {
      if (off[k + 1] == off[k]) { h[0]++; continue; }
      const uint32_t sp = (off[k + 1] - 1) / chunk - off[k] / chunk + 1;
      mx = sp > mx ? sp : mx;
      int b = 1;
      while (b < 11 && sp > (1u << (b - 1))) b++;
      h[b]++;
      if (sp > (sc.cur_sparse ? kSeqSpanSparse : kSeqSpan29) + 1) carries_large += sp; else if (sp > 1) carries_mid += sp;
    }
    fprintf(stderr, "MSMSTATS n=%zu c=%d entries=%u chunk=%u large=%u pieces=%u maxspan=%u carries_mid=%llu "
            "carries_large=%llu spans[empty,1,2,<=4,<=8,..,<=512,>512]=", sc.cur_n, sc.cur_c, M, chunk, cnt, pieces, mx,
            (unsigned long long)carries_mid, (unsigned long long)carries_large);
    for (int b = 0; b < 12; b++) fprintf(stderr, "%zu%c", h[b], b == 11 ? '\n' : ',');
  }
#endif
  const int c = sc.cur_c, nsets = sc.cur_nsets, nslots = sc.cur_nbits + 1;
  if (sc.prof) {
    float t = 0;
    NZ_HIP(hipEventElapsedTime(&t, sc.ev[3], sc.ev[4]));
    // the entry count came with the window sums (msm_enqueue, before `done`): no stream
    // sync here (a sync on the caller's stream waited for whatever followed the MSM on it,
    // e.g. round 1's interpolations behind C's commitment slot: 1.4 ms per proof)
    const uint32_t total = *sc.host_total;
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
  const auto t_host = std::chrono::steady_clock::now();
  struct HostClock {  // the CPU part below, for the phase timing (nzcb_engine_time_msm2)
    MsmScratch& sc;
    std::chrono::steady_clock::time_point t0;
    ~HostClock() {
      if (sc.prof && sc.prof_phases)
        sc.host_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
  } host_clock{sc, t_host};
  if (sc.cur_fixed) return fixed_window_result(sc.host_win, sc.cur_hb, sc.cur_a);  // set 0 (msm_slots29_kernel)
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
