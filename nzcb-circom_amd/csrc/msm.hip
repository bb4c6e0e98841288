// BN254 G1 multi-scalar multiplication for gfx950 (Pippenger, signed windows).
//
// Replaces ffjavascript G1.multiExpAffine + wasmcurves g1m_multiexpAffine_chunk
// (/root/reference/yarn.lock:3905-3913, 8173-8179), which
// split the points into chunks and the scalar bits into pTSizes[log2 n] windows
// (16 bits at 2^21) on CPU workers. The result is a unique group element, so
// any correct schedule is bit-exact after conversion to affine.
//
// Pipeline (one stream, no host sync until the window sums):
//  1. count:      thread per scalar -> signed c-bit digits -> atomic bucket histogram
//  2. scan:       exclusive scan of the histogram (hipCUB) -> bucket offsets
//  3. scatter:    thread per scalar -> point index | sign into its bucket slot
//  4. accumulate: thread per fixed-size chunk of the sorted stream (perfect load
//                 balance whatever the digit distribution); bucket runs fully
//                 inside a chunk are written directly, runs crossing a chunk edge
//                 go to per-chunk carries
//  5. fixup:      the chunk owning a spilling bucket's start folds the carries
//  6. reduce:     per (window, 16-bucket segment) running sums, weighted by the
//                 segment offset; one workgroup per window tree-reduces segments
//  7. host:       Horner over the windows (c doublings each) -> affine
// Bases are read straight from the zkey PTau layout (64 B LEM affine); the
// 2^21-point table is 128 MiB and stays resident in the 256 MiB Infinity Cache
// across the 16 windows' random gathers.
#include "msm.h"

#include <hipcub/hipcub.hpp>
#include <cstdlib>
#include <string>
#include <vector>

namespace nzcb {

static constexpr int kMsmThreads = 256;
static constexpr uint32_t kChunk = 32;
static constexpr int kSegLen = 16;
static constexpr uint32_t kNone = 0xffffffffu;

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

template <int C>
__global__ void __launch_bounds__(kMsmThreads)
msm_count_kernel(const Fr* __restrict__ scalars, size_t n, int mont, uint32_t* __restrict__ counts) {
  constexpr uint32_t NB = 1u << (C - 1);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    Fr s = scalars[i];
    if (mont) s = from_mont(s);
    for_each_digit<C>(s, [&](int w, uint32_t b, uint32_t) { atomicAdd(&counts[w * NB + b], 1u); });
  }
}

template <int C>
__global__ void __launch_bounds__(kMsmThreads)
msm_scatter_kernel(const Fr* __restrict__ scalars, size_t n, int mont, uint32_t* __restrict__ cursor,
                   uint32_t* __restrict__ sorted) {
  constexpr uint32_t NB = 1u << (C - 1);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    Fr s = scalars[i];
    if (mont) s = from_mont(s);
    for_each_digit<C>(s, [&](int w, uint32_t b, uint32_t sign) {
      uint32_t pos = atomicAdd(&cursor[w * NB + b], 1u);
      sorted[pos] = (uint32_t)i | (sign << 31);
    });
  }
}

// Radix-sort path: every (scalar, window) pair gets a fixed slot w*n + i, so no
// atomics are needed; zero digits get the sentinel key nkeys and sort last.
template <int C>
__global__ void __launch_bounds__(kMsmThreads)
msm_keys_kernel(const Fr* __restrict__ scalars, size_t n, int mont, uint32_t* __restrict__ keys,
                uint32_t* __restrict__ vals) {
  constexpr int NW = (255 + C - 1) / C;
  constexpr uint32_t NB = 1u << (C - 1);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    Fr s = scalars[i];
    if (mont) s = from_mont(s);
    uint32_t k[NW];
    uint32_t v[NW];
#pragma unroll
    for (int w = 0; w < NW; w++) {
      k[w] = NW * NB;
      v[w] = (uint32_t)i;
    }
    for_each_digit<C>(s, [&](int w, uint32_t b, uint32_t sign) {
      k[w] = (uint32_t)w * NB + b;
      v[w] = (uint32_t)i | (sign << 31);
    });
#pragma unroll
    for (int w = 0; w < NW; w++) {
      keys[(size_t)w * n + i] = k[w];
      vals[(size_t)w * n + i] = v[w];
    }
  }
}

// offsets[k] = first position of key >= k in the sorted key array (k = 0..nkeys)
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
msm_accumulate_kernel(const G1Affine* __restrict__ bases, const uint32_t* __restrict__ sorted,
                      const uint32_t* __restrict__ offsets, uint32_t nkeys, size_t nthreads,
                      G1xyzz* __restrict__ buckets, G1xyzz* __restrict__ carry_own,
                      G1xyzz* __restrict__ carry_cont, uint32_t* __restrict__ own_key) {
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nthreads) return;
  const uint32_t M = offsets[nkeys];
  const uint32_t s = (uint32_t)t * kChunk;
  if (s >= M) {
    own_key[t] = kNone;
    return;
  }
  const uint32_t e = (s + kChunk < M) ? s + kChunk : M;
  uint32_t k = find_key(offsets, nkeys, s);
  uint32_t kstart = offsets[k], kend = offsets[k + 1];
  G1xyzz acc = G1xyzz::inf();
  uint32_t own = kNone;
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
      else {
        carry_own[t] = acc;
        own = k;
      }
      acc = G1xyzz::inf();
      if (pos < e) {
        k = find_key(offsets, nkeys, pos);
        kstart = offsets[k];
        kend = offsets[k + 1];
      }
    }
  }
  own_key[t] = own;
}

__global__ void __launch_bounds__(kMsmThreads)
msm_fixup_kernel(const uint32_t* __restrict__ offsets, const uint32_t* __restrict__ own_key,
                 const G1xyzz* __restrict__ carry_own, const G1xyzz* __restrict__ carry_cont, size_t nthreads,
                 G1xyzz* __restrict__ buckets) {
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nthreads) return;
  const uint32_t k = own_key[t];
  if (k == kNone) return;
  G1xyzz acc = carry_own[t];
  const uint32_t kend = offsets[k + 1];
  for (size_t u = t + 1; (uint64_t)u * kChunk < kend; u++) acc = xyzz_add(acc, carry_cont[u]);
  buckets[k] = acc;
}

__global__ void __launch_bounds__(kMsmThreads)
msm_bucket_reduce_kernel(const G1xyzz* __restrict__ buckets, const uint32_t* __restrict__ offsets, int nb,
                         int seglen, int nseg, int nw, G1xyzz* __restrict__ seg) {
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)nw * nseg) return;
  const int w = (int)(t / nseg);
  const int g = (int)(t % nseg);
  const size_t base = (size_t)w * nb + (size_t)g * seglen;
  G1xyzz run = G1xyzz::inf(), tot = G1xyzz::inf();
  for (int b = seglen - 1; b >= 0; b--) {
    const size_t key = base + b;
    if (offsets[key + 1] > offsets[key]) run = xyzz_add(run, buckets[key]);
    if (!run.is_inf()) tot = xyzz_add(tot, run);
  }
  // bucket index g*seglen + b carries digit value g*seglen + b + 1
  if (g && !run.is_inf()) tot = xyzz_add(tot, xyzz_mul_small(run, (uint32_t)(g * seglen)));
  seg[t] = tot;
}

__global__ void __launch_bounds__(kMsmThreads)
msm_window_reduce_kernel(const G1xyzz* __restrict__ seg, int nseg, G1xyzz* __restrict__ win) {
  __shared__ G1xyzz sh[kMsmThreads];
  const int w = blockIdx.x;
  G1xyzz acc = G1xyzz::inf();
  for (int i = threadIdx.x; i < nseg; i += blockDim.x) acc = xyzz_add(acc, seg[(size_t)w * nseg + i]);
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int stride = kMsmThreads / 2; stride > 0; stride >>= 1) {
    if ((int)threadIdx.x < stride) sh[threadIdx.x] = xyzz_add(sh[threadIdx.x], sh[threadIdx.x + stride]);
    __syncthreads();
  }
  if (threadIdx.x == 0) win[w] = sh[0];
}

void MsmScratch::init(size_t maxp) {
  max_points = maxp;
  size_t max_entries = 0, max_keys = 0, max_seg = 0;
  for (size_t n = 1;; n <<= 1) {
    size_t m = n < maxp ? n : maxp;
    int c = msm_window_bits(m);
    int nw = num_windows(c);
    size_t nb = size_t(1) << (c - 1);
    size_t seglen = nb < (size_t)kSegLen ? nb : kSegLen;
    max_entries = std::max(max_entries, m * nw);
    max_keys = std::max(max_keys, nb * nw);
    max_seg = std::max(max_seg, (nb / seglen) * nw);
    if (m == maxp) break;
  }
  counts.alloc(max_keys + 1);
  offsets.alloc(max_keys + 1);
  cursor.alloc(max_keys + 1);
  sorted.alloc(max_entries);
  keys_in.alloc(max_entries);
  keys_out.alloc(max_entries);
  vals_in.alloc(max_entries);
  const char* m = std::getenv("NZCB_MSM_SORT");
  use_radix = !(m && std::string(m) == "atomic");
  sort_tmp_bytes = 0;
  NZ_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp_bytes, keys_in.p, keys_out.p, vals_in.p, sorted.p,
                                            max_entries, 0, 21));
  sort_tmp.alloc(sort_tmp_bytes + 16);
  buckets.alloc(max_keys);
  size_t nthreads = (max_entries + kChunk - 1) / kChunk + 1;
  carry_own.alloc(nthreads);
  carry_cont.alloc(nthreads);
  own_key.alloc(nthreads);
  seg.alloc(max_seg);
  win.alloc(64);
  host_win.resize(64);
  scan_tmp_bytes = 0;
  NZ_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tmp_bytes, counts.p, offsets.p, (int)(max_keys + 1)));
  scan_tmp.alloc(scan_tmp_bytes + 16);
}

template <int C>
static void launch_digits(const Fr* scalars, size_t n, int mont, MsmScratch& sc, hipStream_t st, bool scatter) {
  unsigned g = grid_for(n, kMsmThreads, 8192);
  if (sc.use_radix)
    hipLaunchKernelGGL(msm_keys_kernel<C>, dim3(grid_for(n, kMsmThreads, 1u << 30)), dim3(kMsmThreads), 0, st,
                       scalars, n, mont, sc.keys_in.p, sc.vals_in.p);
  else if (!scatter)
    hipLaunchKernelGGL(msm_count_kernel<C>, dim3(g), dim3(kMsmThreads), 0, st, scalars, n, mont, sc.counts.p);
  else
    hipLaunchKernelGGL(msm_scatter_kernel<C>, dim3(g), dim3(kMsmThreads), 0, st, scalars, n, mont, sc.cursor.p,
                       sc.sorted.p);
  NZ_HIP(hipGetLastError());
}

static void digits_dispatch(int c, const Fr* scalars, size_t n, int mont, MsmScratch& sc, hipStream_t st,
                            bool scatter) {
  switch (c) {
#define NZ_CASE(K) case K: launch_digits<K>(scalars, n, mont, sc, st, scatter); break;
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

G1xyzz msm(MsmScratch& sc, const G1Affine* bases, const Fr* scalars, size_t n, bool mont, hipStream_t st) {
  if (n == 0) return G1xyzz::inf();
  if (n > sc.max_points) throw Error(NZCB_ERR_ARG, "msm larger than scratch");
  const int c = msm_window_bits(n);
  const int nw = num_windows(c);
  const uint32_t nb = 1u << (c - 1);
  const uint32_t nkeys = nb * (uint32_t)nw;
  const size_t max_entries = n * (size_t)nw;
  if (sc.use_radix) {
    digits_dispatch(c, scalars, n, mont ? 1 : 0, sc, st, false);
    int end_bit = 1;
    while ((1u << end_bit) <= nkeys) end_bit++;
    size_t tmp = sc.sort_tmp_bytes;
    NZ_HIP(hipcub::DeviceRadixSort::SortPairs(sc.sort_tmp.p, tmp, sc.keys_in.p, sc.keys_out.p, sc.vals_in.p,
                                              sc.sorted.p, max_entries, 0, end_bit, st));
    hipLaunchKernelGGL(msm_offsets_kernel, dim3(grid_for((size_t)nkeys + 1, kMsmThreads, 1u << 30)),
                       dim3(kMsmThreads), 0, st, sc.keys_out.p, max_entries, nkeys, sc.offsets.p);
    NZ_HIP(hipGetLastError());
  } else {
    NZ_HIP(hipMemsetAsync(sc.counts.p, 0, (nkeys + 1) * sizeof(uint32_t), st));
    digits_dispatch(c, scalars, n, mont ? 1 : 0, sc, st, false);
    size_t tmp = sc.scan_tmp_bytes;
    NZ_HIP(hipcub::DeviceScan::ExclusiveSum(sc.scan_tmp.p, tmp, sc.counts.p, sc.offsets.p, (int)(nkeys + 1), st));
    NZ_HIP(hipMemcpyAsync(sc.cursor.p, sc.offsets.p, (nkeys + 1) * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
    digits_dispatch(c, scalars, n, mont ? 1 : 0, sc, st, true);
  }
  const size_t nthreads = (max_entries + kChunk - 1) / kChunk;
  if (sc.prof) {
    if (!sc.ev0) {
      NZ_HIP(hipEventCreate(&sc.ev0));
      NZ_HIP(hipEventCreate(&sc.ev1));
    }
    NZ_HIP(hipEventRecord(sc.ev0, st));
  }
  hipLaunchKernelGGL(msm_accumulate_kernel, dim3(grid_for(nthreads, kMsmThreads, 1u << 30)), dim3(kMsmThreads), 0,
                     st, bases, sc.sorted.p, sc.offsets.p, nkeys, nthreads, sc.buckets.p, sc.carry_own.p,
                     sc.carry_cont.p, sc.own_key.p);
  NZ_HIP(hipGetLastError());
  if (sc.prof) NZ_HIP(hipEventRecord(sc.ev1, st));
  hipLaunchKernelGGL(msm_fixup_kernel, dim3(grid_for(nthreads, kMsmThreads, 1u << 30)), dim3(kMsmThreads), 0, st,
                     sc.offsets.p, sc.own_key.p, sc.carry_own.p, sc.carry_cont.p, nthreads, sc.buckets.p);
  NZ_HIP(hipGetLastError());
  const int seglen = (int)(nb < (uint32_t)kSegLen ? nb : kSegLen);
  const int nseg = (int)(nb / seglen);
  hipLaunchKernelGGL(msm_bucket_reduce_kernel, dim3(grid_for((size_t)nw * nseg, kMsmThreads, 1u << 30)),
                     dim3(kMsmThreads), 0, st, sc.buckets.p, sc.offsets.p, (int)nb, seglen, nseg, nw, sc.seg.p);
  NZ_HIP(hipGetLastError());
  hipLaunchKernelGGL(msm_window_reduce_kernel, dim3(nw), dim3(kMsmThreads), 0, st, sc.seg.p, nseg, sc.win.p);
  NZ_HIP(hipGetLastError());
  NZ_HIP(hipMemcpyAsync(sc.host_win.data(), sc.win.p, nw * sizeof(G1xyzz), hipMemcpyDeviceToHost, st));
  NZ_HIP(hipStreamSynchronize(st));
  if (sc.prof) {
    float t = 0;
    NZ_HIP(hipEventElapsedTime(&t, sc.ev0, sc.ev1));
    uint32_t total = 0;
    NZ_HIP(hipMemcpy(&total, sc.offsets.p + nkeys, 4, hipMemcpyDeviceToHost));
    sc.prof_ms += t;
    sc.prof_launches++;
    sc.prof_points += n;
    sc.prof_entries += total;
  }
  G1xyzz res = G1xyzz::inf();
  for (int w = nw - 1; w >= 0; w--) {
    for (int i = 0; i < c; i++) res = xyzz_dbl(res);
    res = xyzz_add(res, sc.host_win[w]);
  }
  return res;
}

}  // namespace nzcb
