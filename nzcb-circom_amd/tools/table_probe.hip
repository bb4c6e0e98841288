// Random 64-byte gathers against table size (the fixed-base MSM's access pattern):
// does a table of every shifted base 2^e * PTau_i (254 rows, ~34 GB at 2^21) gather as
// fast as today's 15-row table (2 GB)? Address translation is the open question: 2 MB
// pages cover 2 GB in ~1k translations, 34 GB in ~17k.
//   hipcc -O3 --offload-arch=gfx950 table_probe.hip -o table_probe && ./table_probe
// Each kernel gathers 31,457,320 random points (one 2^21-point MSM's entries), 48
// consecutive index slots per thread; the index chunk is staged through LDS first in
// gather64_lds (one coalesced read per wave instead of 48 strided ones per lane).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                     \
  do {                                                            \
    hipError_t e_ = (x);                                          \
    if (e_ != hipSuccess) {                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));     \
      return 1;                                                   \
    }                                                             \
  } while (0)

struct Pt {
  uint4 a, b, c, d;
};

constexpr int kChunk = 48;

__global__ void gather64(const Pt* __restrict__ table, const uint32_t* __restrict__ idx, size_t n,
                         uint32_t* __restrict__ out) {
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t s = t * kChunk;
  if (s >= n) return;
  uint32_t acc = 0;
  for (int i = 0; i < kChunk && s + i < n; i++) {
    const Pt p = table[idx[s + i]];
    acc ^= p.a.x ^ p.a.w ^ p.b.y ^ p.c.z ^ p.d.w ^ p.b.x ^ p.c.y ^ p.d.x;
    acc += p.a.y ^ p.a.z ^ p.b.z ^ p.b.w ^ p.c.x ^ p.c.w ^ p.d.y ^ p.d.z;
  }
  out[t] = acc;
}

__global__ void __launch_bounds__(256) gather64_lds(const Pt* __restrict__ table, const uint32_t* __restrict__ idx,
                                                    size_t n, uint32_t* __restrict__ out) {
  __shared__ uint32_t sidx[256 * kChunk];
  const size_t base = (size_t)blockIdx.x * 256 * kChunk;
  for (int i = threadIdx.x; i < 256 * kChunk; i += 256) sidx[i] = base + i < n ? idx[base + i] : 0u;
  __syncthreads();
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t s = t * kChunk;
  if (s >= n) return;
  uint32_t acc = 0;
  for (int i = 0; i < kChunk && s + i < n; i++) {
    const Pt p = table[sidx[threadIdx.x * kChunk + i]];
    acc ^= p.a.x ^ p.a.w ^ p.b.y ^ p.c.z ^ p.d.w ^ p.b.x ^ p.c.y ^ p.d.x;
    acc += p.a.y ^ p.a.z ^ p.b.z ^ p.b.w ^ p.c.x ^ p.c.w ^ p.d.y ^ p.d.z;
  }
  out[t] = acc;
}

__global__ void fill_idx(uint32_t* idx, size_t n, uint64_t rows, uint64_t seed) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t z = seed + i * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  idx[i] = (uint32_t)(z % rows);
}

int main(int argc, char** argv) {
  const size_t n = 31457320;
  const size_t max_rows = (size_t)1 << 29;  // 32 GiB of 64-byte points
  Pt* table;
  uint32_t *idx, *out;
  CK(hipMalloc(&table, max_rows * sizeof(Pt)));
  CK(hipMalloc(&idx, n * 4));
  CK(hipMalloc(&out, ((size_t)1 << 24) * 4));
  CK(hipMemset(table, 0x5a, max_rows * sizeof(Pt)));
  const size_t threads = (n + kChunk - 1) / kChunk;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int lg = 25; lg <= 29; lg++) {
    const size_t rows = (size_t)1 << lg;
    fill_idx<<<(n + 255) / 256, 256>>>(idx, n, rows, 12345 + lg);
    CK(hipDeviceSynchronize());
    for (int rep = 0; rep < 3; rep++) {
      float ms[2];
      CK(hipEventRecord(e0));
      gather64<<<(threads + 255) / 256, 256>>>(table, idx, n, out);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms[0], e0, e1));
      CK(hipEventRecord(e0));
      gather64_lds<<<(threads + 255) / 256, 256>>>(table, idx, n, out);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms[1], e0, e1));
      printf("table %6.2f GB: gather64 %.3f ms, gather64_lds %.3f ms (%.3f GB of points)\n",
             rows * 64.0 / 1e9, ms[0], ms[1], n * 64.0 / 1e9);
      fflush(stdout);
    }
  }
  CK(hipFree(table));
  CK(hipFree(idx));
  CK(hipFree(out));
  return 0;
}
