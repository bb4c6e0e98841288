// BN254 G1 multi-scalar multiplication for gfx950 (Pippenger, signed windows).
//
// Replaces ffjavascript G1.multiExpAffine + wasmcurves g1m_multiexpAffine_chunk
// (/root/reference/yarn.lock:3905-3913, 8173-8179), which
// split the points into chunks and the scalar bits into pTSizes[log2 n] windows
// (16 bits at 2^21) on CPU workers. The result is a unique group element, so
// any correct schedule is bit-exact after conversion to affine.
//
// Pipeline (one stream, no host sync until the window sums):
//  1. keys:       thread per scalar -> signed c-bit digits; (scalar, window) pair i
//                 gets the fixed slot w*n+i, key = window*2^(c-1) + |digit|-1
//                 (zero digits get a sentinel key that sorts last) -- no atomics
//  2. sort:       rocPRIM radix sort of (key, index|sign) on ceil(log2 keys) bits
//  3. offsets:    bucket start positions by binary search in the sorted keys
//  4. accumulate: thread per fixed 32-entry chunk of the sorted stream (load balance
//                 independent of the digit distribution): XYZZ mixed adds of the
//                 gathered affine bases; bucket runs inside one chunk are written
//                 directly, runs crossing a chunk edge go to per-chunk carries
//  5. reduce:     thread per (window, 16-bucket segment): rebuilds each bucket (one
//                 store or carries) and runs sum/weighted-sum from the top bucket
//  6. sums:       one workgroup per (window, slot): slot 0 sums the segments'
//                 weighted sums, slot b+1 sums the running sums of segments whose
//                 index has bit b set (the segment-offset weights, in binary)
//  7. host:       per window W = T + 16 * sum_b 2^b R_b, then Horner over windows
// Bases are read straight from the zkey PTau layout (64 B LEM affine); the
// 2^21-point table is 128 MiB and stays resident in the 256 MiB Infinity Cache
// across the 16 windows' random gathers.
#include "msm.h"

#include <hipcub/hipcub.hpp>

namespace nzcb {

static constexpr int kMsmThreads = 256;
static constexpr uint32_t kChunk = 32;
static constexpr int kSegLen = 8;

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
msm_accumulate_kernel(const G1Affine* __restrict__ bases, const uint32_t* __restrict__ sorted,
                      const uint32_t* __restrict__ offsets, uint32_t nkeys, size_t nthreads,
                      G1xyzz* __restrict__ buckets, G1xyzz* __restrict__ carry_own,
                      G1xyzz* __restrict__ carry_cont) {
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nthreads) return;
  const uint32_t M = offsets[nkeys];
  const uint32_t s = (uint32_t)t * kChunk;
  if (s >= M) return;
  const uint32_t e = (s + kChunk < M) ? s + kChunk : M;
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

// Kernels below keep exactly one inlined EC addition per loop body: an inlined
// formula is ~3.5k instructions, and several copies in one loop thrash the shared
// instruction cache (measured: 2.7 ms -> see profiles/ for the single-site form).

// Buckets whose entries span several accumulation chunks: owner chunk's carry plus
// the continuation carries of the chunks the bucket spills into (thread per bucket).
__global__ void __launch_bounds__(kMsmThreads)
msm_bucket_finalize_kernel(const uint32_t* __restrict__ offsets, uint32_t nkeys, const G1xyzz* __restrict__ carry_own,
                           const G1xyzz* __restrict__ carry_cont, G1xyzz* __restrict__ buckets) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nkeys) return;
  const uint32_t s = offsets[k], e = offsets[k + 1];
  if (e == s) return;
  const uint32_t c0 = s / kChunk, c1 = (e - 1) / kChunk;
  if (c0 == c1) return;  // the accumulation stored it already
  G1xyzz v = carry_own[c0];
  for (uint32_t u = c0 + 1; u <= c1; u++) v = xyzz_add(v, carry_cont[u]);
  buckets[k] = v;
}

// thread per (window, L-bucket segment): run = sum_j B_j, tot = sum_j (j+1) B_j
__global__ void __launch_bounds__(kMsmThreads)
msm_bucket_reduce_kernel(const G1xyzz* __restrict__ buckets, const uint32_t* __restrict__ offsets, int nb,
                         int seglen, int nseg, int nw, G1xyzz* __restrict__ seg_tot, G1xyzz* __restrict__ seg_run) {
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)nw * nseg) return;
  const int w = (int)(t / nseg);
  const int g = (int)(t % nseg);
  const size_t base = (size_t)w * nb + (size_t)g * seglen;
  G1xyzz run = G1xyzz::inf(), tot = G1xyzz::inf();
  for (int st = 0; st < 2 * seglen; st++) {
    const bool is_run = !(st & 1);
    G1xyzz rhs;
    if (is_run) {
      const uint32_t k = (uint32_t)(base + seglen - 1 - (st >> 1));
      if (offsets[k + 1] == offsets[k]) continue;
      rhs = buckets[k];
    } else {
      if (run.is_inf()) continue;
      rhs = run;
    }
    const G1xyzz r = xyzz_add(is_run ? run : tot, rhs);
    if (is_run) run = r; else tot = r;
  }
  seg_tot[t] = tot;  // sum_j (j+1) * bucket_{g*L+j}
  seg_run[t] = run;  // sum_j bucket_{g*L+j}
}

// workgroup (w, j): j = 0 -> sum_g seg_tot[w][g]; j = b+1 -> sum of seg_run[w][g] over g with bit b set
__global__ void __launch_bounds__(kMsmThreads)
msm_window_sums_kernel(const G1xyzz* __restrict__ seg_tot, const G1xyzz* __restrict__ seg_run, int nseg,
                       int nslots, G1xyzz* __restrict__ out) {
  __shared__ G1xyzz sh[kMsmThreads];
  const int w = blockIdx.x / nslots;
  const int j = blockIdx.x % nslots;
  const int tid = threadIdx.x;
  const int count = j == 0 ? nseg : nseg >> 1;
  const int nacc = (count + kMsmThreads - 1) / kMsmThreads;
  int lg = 0;
  while ((1 << lg) < kMsmThreads) lg++;
  G1xyzz acc = G1xyzz::inf();
  for (int step = 0; step < nacc + lg; step++) {
    if (step == nacc) {
      sh[tid] = acc;
      __syncthreads();
    }
    bool doit;
    G1xyzz lhs, rhs;
    if (step < nacc) {
      const int q = tid + step * kMsmThreads;
      doit = q < count;
      if (doit) {
        int g = q;
        if (j) {
          const int b = j - 1;
          g = ((q >> b) << (b + 1)) | (1 << b) | (q & ((1 << b) - 1));
        }
        rhs = j ? seg_run[(size_t)w * nseg + g] : seg_tot[(size_t)w * nseg + g];
        lhs = acc;
      }
    } else {
      const int stride = (kMsmThreads >> 1) >> (step - nacc);
      doit = tid < stride;
      if (doit) {
        lhs = sh[tid];
        rhs = sh[tid + stride];
      }
    }
    G1xyzz r;
    if (doit) r = xyzz_add(lhs, rhs);
    if (step < nacc) {
      if (doit) acc = r;
    } else {
      if (doit) sh[tid] = r;
      __syncthreads();
    }
  }
  if (tid == 0) out[blockIdx.x] = sh[0];
}

static void msm_shape(size_t n, int& c, int& nw, uint32_t& nb, int& seglen, int& nseg, int& nbits) {
  c = msm_window_bits(n);
  nw = num_windows(c);
  nb = 1u << (c - 1);
  seglen = (int)(nb < (uint32_t)kSegLen ? nb : kSegLen);
  nseg = (int)(nb / seglen);
  nbits = 0;
  while ((1 << nbits) < nseg) nbits++;
}

void MsmScratch::init(size_t maxp) {
  max_points = maxp;
  size_t max_entries = 0, max_keys = 0, max_seg = 0, max_slots = 0;
  for (size_t n = 1;; n <<= 1) {
    size_t m = n < maxp ? n : maxp;
    int c, nw, seglen, nseg, nbits;
    uint32_t nb;
    msm_shape(m, c, nw, nb, seglen, nseg, nbits);
    max_entries = std::max(max_entries, m * nw);
    max_keys = std::max(max_keys, (size_t)nb * nw);
    max_seg = std::max(max_seg, (size_t)nseg * nw);
    max_slots = std::max(max_slots, (size_t)(nbits + 1) * nw);
    if (m == maxp) break;
  }
  offsets.alloc(max_keys + 1);
  sorted.alloc(max_entries);
  keys_in.alloc(max_entries);
  keys_out.alloc(max_entries);
  vals_in.alloc(max_entries);
  sort_tmp_bytes = 0;
  NZ_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp_bytes, keys_in.p, keys_out.p, vals_in.p, sorted.p,
                                            max_entries, 0, 21));
  sort_tmp.alloc(sort_tmp_bytes + 16);
  buckets.alloc(max_keys);
  size_t nthreads = (max_entries + kChunk - 1) / kChunk + 1;
  carry_own.alloc(nthreads);
  carry_cont.alloc(nthreads);
  seg_tot.alloc(max_seg);
  seg_run.alloc(max_seg);
  win.alloc(max_slots);
  host_win_cap = max_slots;
  NZ_HIP(hipHostMalloc((void**)&host_win, max_slots * sizeof(G1xyzz), hipHostMallocDefault));
}

MsmScratch::~MsmScratch() {
  if (host_win) (void)hipHostFree(host_win);
  if (ev0) (void)hipEventDestroy(ev0);
  if (ev1) (void)hipEventDestroy(ev1);
}

template <int C>
static void launch_keys(const Fr* scalars, size_t n, int mont, MsmScratch& sc, hipStream_t st) {
  hipLaunchKernelGGL(msm_keys_kernel<C>, dim3(grid_for(n, kMsmThreads, 1u << 30)), dim3(kMsmThreads), 0, st,
                     scalars, n, mont, sc.keys_in.p, sc.vals_in.p);
  NZ_HIP(hipGetLastError());
}

static void keys_dispatch(int c, const Fr* scalars, size_t n, int mont, MsmScratch& sc, hipStream_t st) {
  switch (c) {
#define NZ_CASE(K) case K: launch_keys<K>(scalars, n, mont, sc, st); break;
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

void msm_enqueue(MsmScratch& sc, const G1Affine* bases, const Fr* scalars, size_t n, bool mont, hipStream_t st) {
  sc.cur_n = n;
  if (n == 0) return;
  if (n > sc.max_points) throw Error(NZCB_ERR_ARG, "msm larger than scratch");
  int c, nw, seglen, nseg, nbits;
  uint32_t nb;
  msm_shape(n, c, nw, nb, seglen, nseg, nbits);
  const uint32_t nkeys = nb * (uint32_t)nw;
  sc.cur_c = c;
  sc.cur_nw = nw;
  sc.cur_nbits = nbits;
  sc.cur_seglen = seglen;
  sc.cur_nkeys = nkeys;
  const size_t entries = n * (size_t)nw;
  keys_dispatch(c, scalars, n, mont ? 1 : 0, sc, st);
  int end_bit = 1;
  while ((1u << end_bit) <= nkeys) end_bit++;
  size_t tmp = sc.sort_tmp_bytes;
  NZ_HIP(hipcub::DeviceRadixSort::SortPairs(sc.sort_tmp.p, tmp, sc.keys_in.p, sc.keys_out.p, sc.vals_in.p,
                                            sc.sorted.p, entries, 0, end_bit, st));
  hipLaunchKernelGGL(msm_offsets_kernel, dim3(grid_for((size_t)nkeys + 1, kMsmThreads, 1u << 30)), dim3(kMsmThreads),
                     0, st, sc.keys_out.p, entries, nkeys, sc.offsets.p);
  NZ_HIP(hipGetLastError());
  const size_t nthreads = (entries + kChunk - 1) / kChunk;
  if (sc.prof) {
    if (!sc.ev0) {
      NZ_HIP(hipEventCreate(&sc.ev0));
      NZ_HIP(hipEventCreate(&sc.ev1));
    }
    NZ_HIP(hipEventRecord(sc.ev0, st));
  }
  hipLaunchKernelGGL(msm_accumulate_kernel, dim3(grid_for(nthreads, kMsmThreads, 1u << 30)), dim3(kMsmThreads), 0,
                     st, bases, sc.sorted.p, sc.offsets.p, nkeys, nthreads, sc.buckets.p, sc.carry_own.p,
                     sc.carry_cont.p);
  NZ_HIP(hipGetLastError());
  if (sc.prof) NZ_HIP(hipEventRecord(sc.ev1, st));
  hipLaunchKernelGGL(msm_bucket_finalize_kernel, dim3(grid_for(nkeys, kMsmThreads, 1u << 30)), dim3(kMsmThreads), 0,
                     st, sc.offsets.p, nkeys, sc.carry_own.p, sc.carry_cont.p, sc.buckets.p);
  NZ_HIP(hipGetLastError());
  hipLaunchKernelGGL(msm_bucket_reduce_kernel, dim3(grid_for((size_t)nw * nseg, kMsmThreads, 1u << 30)),
                     dim3(kMsmThreads), 0, st, sc.buckets.p, sc.offsets.p, (int)nb, seglen, nseg, nw, sc.seg_tot.p,
                     sc.seg_run.p);
  NZ_HIP(hipGetLastError());
  const int nslots = nbits + 1;
  hipLaunchKernelGGL(msm_window_sums_kernel, dim3(nw * nslots), dim3(kMsmThreads), 0, st, sc.seg_tot.p, sc.seg_run.p,
                     nseg, nslots, sc.win.p);
  NZ_HIP(hipGetLastError());
  NZ_HIP(hipMemcpyAsync(sc.host_win, sc.win.p, (size_t)nw * nslots * sizeof(G1xyzz), hipMemcpyDeviceToHost, st));
}

G1xyzz msm_finish(MsmScratch& sc, hipStream_t st) {
  if (sc.cur_n == 0) return G1xyzz::inf();
  NZ_HIP(hipStreamSynchronize(st));
  const int c = sc.cur_c, nw = sc.cur_nw, nslots = sc.cur_nbits + 1;
  if (sc.prof) {
    float t = 0;
    NZ_HIP(hipEventElapsedTime(&t, sc.ev0, sc.ev1));
    uint32_t total = 0;
    NZ_HIP(hipMemcpy(&total, sc.offsets.p + sc.cur_nkeys, 4, hipMemcpyDeviceToHost));
    sc.prof_ms += t;
    sc.prof_launches++;
    sc.prof_points += sc.cur_n;
    sc.prof_entries += total;
  }
  int lg_seg = 0;
  while ((1 << lg_seg) < sc.cur_seglen) lg_seg++;
  G1xyzz res = G1xyzz::inf();
  for (int w = nw - 1; w >= 0; w--) {
    const G1xyzz* s = sc.host_win + (size_t)w * nslots;
    // sum_g g * run_g = sum_b 2^b R_b  (Horner over the bits), times the segment length
    G1xyzz acc = G1xyzz::inf();
    for (int b = nslots - 2; b >= 0; b--) {
      acc = xyzz_dbl(acc);
      acc = xyzz_add(acc, s[1 + b]);
    }
    for (int i = 0; i < lg_seg; i++) acc = xyzz_dbl(acc);
    const G1xyzz W = xyzz_add(acc, s[0]);
    for (int i = 0; i < c; i++) res = xyzz_dbl(res);
    res = xyzz_add(res, W);
  }
  return res;
}

}  // namespace nzcb
