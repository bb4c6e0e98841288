// Fr NTT for gfx950: LDS-tiled radix-2 passes, up to 8 stages per HBM round trip.
//
// Replaces ffjavascript Fr.fft / Fr.ifft (wasmcurves frm_fftMix / fftJoin /
// fftFinal). Semantics: natural order in and out,
// fft: A[i] = sum_j a[j] w^(ij); ifft: a[j] = N^-1 sum_i A[i] w^(-ij), w = w[log2 N].
//
// Plan for N = 2^L (DIT): pass 0 gathers 2^q-element blocks in bit-reversed
// order (bit reversal fused into the load: a tile is 2^q rows x C consecutive
// columns, so every row load is C*32 contiguous bytes) and runs stages 0..q-1
// in LDS; later passes run stages s..s+q-1 on tiles of 2^q rows (stride 2^s)
// x C consecutive columns, in place. L = 23 -> 3 passes of <= 8 stages, each one
// read + one write of the array (algorithmic 64 B per element per pass).
//
// The pass is bound by Montgomery products (one per butterfly), so the kernel is
// shaped for issue rate: 256 threads per 1024-element tile (4 tiles per CU -> 4 waves
// per SIMD), stages are done two at a time as radix-4 groups held in registers
// (4 elements per thread: half the LDS traffic and barriers of radix-2), twiddles
// come from per-stage compact tables (consecutive butterflies -> consecutive
// twiddles), and stage 0's unit twiddles are skipped.
#include "ntt.h"

#include <vector>

namespace nzcb {

static constexpr int kTile = 1024;  // elements per LDS tile: 9 x 4 KiB of 29-bit limbs, 256 threads

Fr fr_root_of_unity(int k) {
  Fr w;
  const uint32_t w28[8] = {0x725b19f0u, 0x9bd61b6eu, 0x41112ed4u, 0x402d111eu,
                           0x8ef62abcu, 0x00e0a7ebu, 0xa58a7e85u, 0x2a3c09f0u};
  for (int i = 0; i < 8; i++) w.v[i] = w28[i];
  w = to_mont(w);
  for (int j = 28; j > k; j--) w = sqr(w);
  return w;
}

__device__ __forceinline__ uint32_t bit_rev(uint32_t x, int bits) {
  return bits ? (__brev(x) >> (32 - bits)) : 0u;
}

// full[i] = lo[i & 2047] * hi[i >> 11] = W^i for i < 2^(L-1)
__global__ void __launch_bounds__(256)
ntt_table_kernel(Fr* __restrict__ out, const Fr* __restrict__ lo, const Fr* __restrict__ hi, size_t count) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  out[i] = lo[i & 2047] * hi[i >> 11];
}

// compact[2^g - 1 + k] = full[k << (L - g - 1)], g < L, k < 2^g
__global__ void __launch_bounds__(256)
ntt_stage_table_kernel(Fr* __restrict__ out, const Fr* __restrict__ full, int L, size_t count) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  int g = 63 - __clzll((unsigned long long)(i + 1));  // i + 1 in [2^g, 2^(g+1))
  size_t k = i + 1 - ((size_t)1 << g);
  out[i] = full[k << (L - g - 1)];
}

// the Shoup operand pair of a twiddle given in Montgomery-256 form (s = w 2^256 mod r):
// w = from_mont(s), and ws = floor(w 2^261 / r) from m = w 2^261 mod r (= s 2^5 mod r):
// w 2^261 = ws r + m, so ws = -m r^-1 mod 2^261 (exact; ws < 2^261), a low-half product
__global__ void __launch_bounds__(256) ntt_tw29_kernel(NttTables::Tw* __restrict__ out, const Fr* __restrict__ tw,
                                                       size_t count) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  Fr m = tw[i];
#pragma unroll
  for (int k = 0; k < 5; k++) m = m + m;
  NttTables::Tw t;
  t.w = split29(from_mont(tw[i]));
  t.ws = mul_lo261(split29(m), f29_const(Fr29::NINV));
  out[i] = t;
}

void NttTables::init(int L, hipStream_t st) {
  max_log = L;
  if (L > 8) scratch29.alloc((size_t)9 << L);  // the 9x29 pipeline's inter-pass values
  const size_t half = L >= 1 ? (size_t(1) << (L - 1)) : 1;
  const size_t total = (size_t(1) << L) - 1;
  DevBuf<Fr> stage(total ? total : 1);  // one direction's Montgomery-256 stage table
  fwd29.alloc(total ? total : 1);
  inv29.alloc(total ? total : 1);
  DevBuf<Fr> full(half);
  for (int dir = 0; dir < 2; dir++) {
    Fr w = fr_root_of_unity(L);
    if (dir) w = inverse(w);
    size_t nlo = half < 2048 ? half : 2048;
    size_t nhi = (half + 2047) / 2048;
    std::vector<Fr> lo(2048, Fr::one()), hi(nhi, Fr::one());
    for (size_t i = 1; i < nlo; i++) lo[i] = lo[i - 1] * w;
    Fr w2048 = pow_u64(w, 2048);
    for (size_t i = 1; i < nhi; i++) hi[i] = hi[i - 1] * w2048;
    DevBuf<Fr> dlo(2048), dhi(nhi);
    NZ_HIP(hipMemcpyAsync(dlo.p, lo.data(), 2048 * sizeof(Fr), hipMemcpyHostToDevice, st));
    NZ_HIP(hipMemcpyAsync(dhi.p, hi.data(), nhi * sizeof(Fr), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(ntt_table_kernel, dim3(grid_for(half, 256, 1u << 30)), dim3(256), 0, st, full.p, dlo.p, dhi.p,
                       half);
    if (total) {
      hipLaunchKernelGGL(ntt_stage_table_kernel, dim3(grid_for(total, 256, 1u << 30)), dim3(256), 0, st,
                         stage.p, full.p, L, total);
      hipLaunchKernelGGL(ntt_tw29_kernel, dim3(grid_for(total, 256, 1u << 30)), dim3(256), 0, st,
                         dir ? inv29.p : fwd29.p, stage.p, total);
    }
    NZ_HIP(hipGetLastError());
    NZ_HIP(hipStreamSynchronize(st));
  }
}

// ---- 9x29-bit pipeline ----------------------------------------------------------------
// The transform's values stay in the redundant radix 2^29 of f29.h from the first pass's
// load to the last pass's store: LDS tiles, registers and the inter-pass HBM scratch hold
// 9 x 29-bit limbs, so a butterfly is one twiddle product plus limb adds.
// Twiddle products (round 5) are Shoup products by the fixed twiddle (f29.h mul_shoup: 143
// mads and no v_mul_lo_u32 against the Montgomery product's 162 + 9; NttTables::Tw holds
// w and floor(w 2^261 / r)). Bounds (r = the BN254 scalar modulus):
//  * a twiddle product of x < 2^261 (limbs < 2^30.7) is < 3r, limbs normalized;
//  * a butterfly y0 = x0 + t, y1 = x0 + 4r - t (Fr29::K4 borrowed: every limb, the top one
//    included, >= t's) adds at most 4r to the value bound of its inputs, so after the L <= 24
//    stages of a transform from inputs < 2.4 r the values are < 99 r < 2^260.3 (every
//    product input < 2^261 holds throughout, no value reduction is ever needed);
//  * limbs: a radix-4 group's outputs are < 2^31.3 before normalisation, its products'
//    inputs < 2^30.7; the outputs are normalized (norm29) once per group (and after the
//    odd radix-2 stage), so every group starts from limbs < 2^29;
//  * the last pass maps v < 128 r to canonical Fr: q = floor(v_8 / (r_8 + 1)) <= v / r
//    (v_8 = the top limb, bits 232..), v - q r < r + (q + 1) 2^232 < 2r, then one
//    conditional subtraction (join_fr29); with an output factor (a Montgomery product by
//    the per-index out_f) the product < x r / 2^261 + r < 1.6 r is joined directly.
// Until round 4 the twiddles were Montgomery-261 operands of mul29 (products < 1.4 r,
// butterflies + 2r, values < 50 r).
// elements per tile: 1024 (9 x 4 KiB of limbs = 36 KiB LDS, 256 threads, 4 tiles per CU), one
// radix-4 group per thread; 2048-element tiles (72 KiB, 2 per CU) give the same 4 waves per
// SIMD in half as many barrier domains and measured slower (profiles/r3_ntt_tile_ab.txt)

// LDS slot of tile element e: bits 0-4 XORed with a function of bits 5-7, a bijection on
// every 32-element block. ds_read_b32 / ds_write_b32 bank by (address / 4) mod 32 per
// 32-lane half, and with 8-column tiles (logC = 3) the first pass's transposed store
// (element stride 8) hit 4 banks (8-way) and the radix-4 step at stage 0 (row stride 4,
// element stride 32) 8 banks (4-way); swizzled, every access pattern of the kernel
// (row-major loads/stores, all radix-4 operand sets at each stage, the odd radix-2
// stage, the sparse copy) is conflict-free (checked exhaustively for q = 6, 7, 8).
__device__ __forceinline__ int tile_slot(int e) {
  return e ^ ((((e >> 5) & 3) << 3) | ((e >> 5) & 7));
}
__device__ __forceinline__ F29 tile_ld(const uint32_t* sl, int e) {
  const int p = tile_slot(e);
  F29 x;
#pragma unroll
  for (int l = 0; l < 9; l++) x.v[l] = sl[l * kTile + p];
  return x;
}
__device__ __forceinline__ void tile_st(uint32_t* sl, int e, const F29& x) {
  const int p = tile_slot(e);
#pragma unroll
  for (int l = 0; l < 9; l++) sl[l * kTile + p] = x.v[l];
}
__device__ __forceinline__ F29 add_nn29(const F29& a, const F29& b) {
  F29 r;
#pragma unroll
  for (int l = 0; l < 9; l++) r.v[l] = a.v[l] + b.v[l];
  return r;
}
// twiddle products (Shoup, f29.h): one, and two interleaved
__device__ __forceinline__ F29 tw_mul(const F29& x, const NttTables::Tw& w) { return mul_shoup(x, w.w, w.ws); }
__device__ __forceinline__ void tw_mul2(const F29& x, const NttTables::Tw& w, const F29& y, const NttTables::Tw& v,
                                        F29& r1, F29& r2) {
  mul_shoup_x2(x, w.w, w.ws, y, v.w, v.ws, r1, r2);
}
__device__ __forceinline__ F29 sub4r_nn29(const F29& a, const F29& b) {  // a + 4r - b, b < 3r normalized
  F29 r;
#pragma unroll
  for (int l = 0; l < 9; l++) r.v[l] = a.v[l] + Fr29::K4[l] - b.v[l];
  return r;
}

// One pass of stages [s, s+q) on tiles of (2^q rows) x (2^logC columns). IN29: values from
// the F29 scratch (else the Fr input, first pass only); OUT29: values to the F29 scratch
// (else canonical Fr to `out`, last pass only).
template <bool IN29, bool OUT29>
__global__ void __launch_bounds__(kTile / 4)
ntt29_pass_kernel(const Fr* in, const F29* in29, Fr* out, F29* out29, const NttTables::Tw* __restrict__ tw, int L, int s,
                  int q, int logC, F29 scale29, int do_scale, NttIo io, int sparse4) {
  constexpr int T = kTile / 4;  // threads
  __shared__ uint32_t sl[9 * kTile];
  const int C = 1 << logC;
  const int rows = 1 << q;
  const int n_el = rows << logC;
  const int tid = threadIdx.x;
  const size_t t = blockIdx.x;
  size_t base = 0, c0 = 0, lo0 = 0;
  if (!IN29) {  // first pass: bit-reversed gather of the Fr input, prologue factors
    c0 = t << logC;
    for (int e = tid; e < n_el; e += T) {
      const int j = e >> logC, c = e & (C - 1);
      const size_t src = ((size_t)bit_rev((uint32_t)j, q) << (L - q)) + c0 + c;
      F29 x;
#pragma unroll
      for (int l = 0; l < 9; l++) x.v[l] = 0;
      if (src < io.in_len) {
        x = split29(in[src]);
        if (src < io.fold_len) {  // + in[src + n] d: limbs < 2^30, value < 2.4 r (mul29 inputs)
          const F29 hi = mul29<Fr29>(split29(in[src + io.fold_n]), io.fold_f);
#pragma unroll
          for (int l = 0; l < 9; l++) x.v[l] += hi.v[l];
          if (!io.in_f) {
            norm29(x);
            x = split29(canon_fr29(x));
          }
        }
        if (io.in_f) x = mul29<Fr29>(x, io.in_f[src]);
        if (do_scale) x = mul29<Fr29>(x, scale29);
      }
      tile_st(sl, e, x);
    }
  } else {
    const size_t groups_lo = ((size_t)1 << s) >> logC;
    const size_t hi = t / groups_lo;
    lo0 = (t % groups_lo) << logC;
    base = (hi << (s + q)) + lo0;
    for (int e = tid; e < n_el; e += T) {
      const int j = e >> logC, c = e & (C - 1);
      tile_st(sl, e, in29[base + ((size_t)j << s) + c]);
    }
  }
  __syncthreads();
  const int nbf = n_el >> 1;
  const bool first = !IN29;
  int st = 0;
  if (sparse4 && blockIdx.x != 0) {
    // zero-padded input past tile 0: of every four bit-reversed rows 4m..4m+3 only row 4m
    // is nonzero, and stages 0-1 map (x, 0, 0, 0) to (x, x, x, x): the first radix-4 step
    // is a copy
    for (int e = tid; e < n_el; e += T) {
      const int j = e >> logC;
      if (j & 3) tile_st(sl, e, tile_ld(sl, ((j & ~3) << logC) + (e & (C - 1))));
    }
    __syncthreads();
    st = 2;
  } else if (q & 1) {  // odd stage count: one radix-2 stage first
    const int g = s;
    const NttTables::Tw* __restrict__ twg = tw + (((size_t)1 << g) - 1);
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const int b = tid + u * T;
      if (b >= nbf) continue;
      const int c = b & (C - 1);
      const int j0 = b >> logC;
      const int i0 = ((2 * j0) << logC) + c, i1 = ((2 * j0 + 1) << logC) + c;
      const size_t k = first ? 0 : (lo0 + c);
      const F29 x0 = tile_ld(sl, i0);
      const F29 x1 = tile_ld(sl, i1);
      const F29 tt = g ? tw_mul(x1, twg[k]) : x1;
      F29 y0 = add_nn29(x0, tt), y1 = sub4r_nn29(x0, tt);
      norm29(y0);
      norm29(y1);
      tile_st(sl, i0, y0);
      tile_st(sl, i1, y1);
    }
    __syncthreads();
    st = 1;
  }
  const int ngroups = n_el >> 2;
#pragma unroll 1
  for (; st < q; st += 2) {
    const int h = 1 << st;
    const int g = s + st;
    const NttTables::Tw* __restrict__ twa = tw + (((size_t)1 << g) - 1);
    const NttTables::Tw* __restrict__ twb = tw + (((size_t)1 << (g + 1)) - 1);
    const int b = tid;
    if (b < ngroups) {
      const int c = b & (C - 1);
      const int pr = b >> logC;
      const int low = pr & (h - 1);
      const int j = ((pr >> st) << (st + 2)) | low;
      const size_t ka = first ? (size_t)low : (((size_t)low << s) + lo0 + c);
      const size_t kc = first ? (size_t)(low + h) : (((size_t)(low + h) << s) + lo0 + c);
      const int i0 = (j << logC) + c, i1 = ((j + h) << logC) + c, i2 = ((j + 2 * h) << logC) + c,
                i3 = ((j + 3 * h) << logC) + c;
      F29 t1 = tile_ld(sl, i1), t3 = tile_ld(sl, i3);
      if (g) {
        const NttTables::Tw wa = twa[ka];
        F29 p1, p3;
        tw_mul2(t1, wa, t3, wa, p1, p3);
        t1 = p1;
        t3 = p3;
      }
      const F29 x0 = tile_ld(sl, i0), x2 = tile_ld(sl, i2);
      const F29 y0 = add_nn29(x0, t1), y1 = sub4r_nn29(x0, t1);
      const F29 y2 = add_nn29(x2, t3), y3 = sub4r_nn29(x2, t3);
      F29 u2, u3;
      const NttTables::Tw wb = twb[ka], wc = twb[kc];
      tw_mul2(y2, wb, y3, wc, u2, u3);
      F29 z0 = add_nn29(y0, u2), z2 = sub4r_nn29(y0, u2), z1 = add_nn29(y1, u3), z3 = sub4r_nn29(y1, u3);
      norm29(z0);
      norm29(z1);
      norm29(z2);
      norm29(z3);
      tile_st(sl, i0, z0);
      tile_st(sl, i1, z1);
      tile_st(sl, i2, z2);
      tile_st(sl, i3, z3);
    }
    __syncthreads();
  }
  auto store = [&](size_t dst, const F29& x) {
    if (OUT29) {
      out29[dst] = x;
    } else {
      const Fr v = io.out_f ? join_fr29(mul29<Fr29>(x, io.out_f[dst])) : canon_fr29(x);
      if (io.out_flags && dst >= io.out_limit && !v.is_zero()) atomicOr(io.out_flags, 1u);
      out[dst] = v;
    }
  };
  if (first) {
    for (int e = tid; e < n_el; e += T) {
      const int j = e & (rows - 1), c = e >> q;
      const size_t dst = ((size_t)bit_rev((uint32_t)(c0 + c), L - q) << q) + j;
      store(dst, tile_ld(sl, (j << logC) + c));
    }
  } else {
    for (int e = tid; e < n_el; e += T) {
      const int j = e >> logC, c = e & (C - 1);
      store(base + ((size_t)j << s) + c, tile_ld(sl, e));
    }
  }
}

// The 9x29 pipeline's passes: stages [0, q1) with the bit-reversed gather, then <= 8
// stages per pass through the F29 scratch; the last pass writes canonical Fr.
static void ntt29_passes(const Fr* in, Fr* out, const NttTables::Tw* tw, int L, const F29& sc29, int do_scale,
                         const NttIo& io, hipStream_t st, F29* scr) {
  constexpr int T = kTile / 4;
  const int q1 = L < 8 ? L : 8;
  const int cols = 1 << (L - q1);
  int logC1 = 0;
  while ((1 << (logC1 + 1)) <= cols && ((1 << (q1 + logC1 + 1)) <= kTile)) logC1++;
  const size_t tiles = (size_t)cols >> logC1;
  // inputs nonzero only below N/4 (+ a few in tile 0's columns: the blinding terms):
  // tiles past the first skip stages 0-1 (a 4n coset NTT of an n+3-term polynomial)
  const int sparse4 = L >= 2 && q1 >= 2 && !(q1 & 1) &&
                      io.in_len <= ((size_t)1 << (L - 2)) + ((size_t)1 << logC1);
  if (q1 == L) {
    hipLaunchKernelGGL((ntt29_pass_kernel<false, false>), dim3((unsigned)tiles), dim3(T), 0, st, in,
                       (const F29*)nullptr, out, (F29*)nullptr, tw, L, 0, q1, logC1, sc29, do_scale, io, sparse4);
    NZ_HIP(hipGetLastError());
    return;
  }
  hipLaunchKernelGGL((ntt29_pass_kernel<false, true>), dim3((unsigned)tiles), dim3(T), 0, st, in,
                     (const F29*)nullptr, (Fr*)nullptr, scr, tw, L, 0, q1, logC1, sc29, do_scale, io, sparse4);
  NZ_HIP(hipGetLastError());
  int s = q1;
  while (s < L) {
    const int q = (L - s) < 8 ? (L - s) : 8;
    int logC = 0;
    while (logC + 1 <= s && (1 << (q + logC + 1)) <= kTile) logC++;
    const size_t ntiles = ((size_t)1 << (L - s - q)) * (((size_t)1 << s) >> logC);
    if (s + q == L)
      hipLaunchKernelGGL((ntt29_pass_kernel<true, false>), dim3((unsigned)ntiles), dim3(T), 0, st,
                         (const Fr*)nullptr, (const F29*)scr, out, (F29*)nullptr, tw, L, s, q, logC, sc29, 0, io, 0);
    else
      hipLaunchKernelGGL((ntt29_pass_kernel<true, true>), dim3((unsigned)ntiles), dim3(T), 0, st,
                         (const Fr*)nullptr, (const F29*)scr, (Fr*)nullptr, scr, tw, L, s, q, logC, sc29, 0, io, 0);
    NZ_HIP(hipGetLastError());
    s += q;
  }
}

void ntt(const NttTables& t, const Fr* in, Fr* out, int L, bool inverse_dir, hipStream_t st, const Fr* scale,
         const NttIo* iop, uint32_t* scratch29) {
  const NttIo io = iop ? *iop : NttIo();
  if (L > t.max_log) throw Error(NZCB_ERR_ARG, "ntt size exceeds table");
  if (in == out) throw Error(NZCB_ERR_ARG, "ntt requires in != out");
  F29* scr = (F29*)(scratch29 ? scratch29 : t.scratch29.p);
  if (L > 8 && !scratch29 && t.scratch29.n < ((size_t)9 << L)) throw Error(NZCB_ERR_INTERNAL, "ntt: no scratch");
  const NttTables::Tw* tw = inverse_dir ? t.inv29.p : t.fwd29.p;
  Fr sc = Fr::one();
  int do_scale = 0;
  if (inverse_dir && !io.out_f_has_scale) {
    Fr two = Fr::one() + Fr::one();
    sc = inverse(pow_u64(two, (uint64_t)L));  // N^-1
    do_scale = 1;
  }
  if (scale) {
    sc = do_scale ? sc * *scale : *scale;
    do_scale = 1;
  }
  for (int k = 0; k < 5; k++) sc = sc + sc;  // Montgomery-261 operand of mul_fr29
  ntt29_passes(in, out, tw, L, split29(sc), do_scale, io, st, scr);
}

}  // namespace nzcb
