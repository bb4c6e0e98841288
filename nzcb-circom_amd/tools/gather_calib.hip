// FETCH_SIZE calibration for the MSM accumulation's access pattern:
// known byte counts, read through rocprofv3 --pmc FETCH_SIZE, give the factor between
// the counter and the bytes actually fetched for
//   kernel gather64  : each lane loads random 64-byte affine points (G1Affine, as
//                      msm_accumulate29_kernel does: 4 x 16-byte loads per point) from a
//                      2 GiB table, 32 consecutive index slots per thread (the chunk)
//   kernel stream16  : the guide's reference case, a coalesced 16 B/lane streaming read
//                      of the same 2 GiB (MI355X_MICROARCH.md: FETCH_SIZE = 1/2 of the bytes)
//   kernel idx_only  : the 4-byte index stream alone (subtracted from gather64)
// Both tables are far past the 256 MiB Infinity Cache, so nothing is served on-die.
//   hipcc -O3 --offload-arch=gfx950 gather_calib.hip -o gather_calib
//   rocprofv3 --pmc FETCH_SIZE -d out -o run --output-format csv -- ./gather_calib
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      return 1;                                                                \
    }                                                                          \
  } while (0)

struct Pt {
  uint4 a, b, c, d;  // 64 bytes, like G1Affine (x||y, 8 limbs each)
};

constexpr int kChunk = 32;

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

__global__ void idx_only(const uint32_t* __restrict__ idx, size_t n, uint32_t* __restrict__ out) {
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t s = t * kChunk;
  if (s >= n) return;
  uint32_t acc = 0;
  for (int i = 0; i < kChunk && s + i < n; i++) acc += idx[s + i] * 2654435761u;
  out[t] = acc;
}

__global__ void stream16(const uint4* __restrict__ src, size_t n16, uint32_t* __restrict__ out) {
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (size_t i = t; i < n16; i += stride) {
    uint4 v = src[i];
    acc ^= v.x + v.y + v.z + v.w;
  }
  out[t] = acc;
}

__global__ void fill_idx(uint32_t* idx, size_t n, uint32_t rows, uint64_t seed) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t z = seed + i * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  idx[i] = (uint32_t)(z % rows);
}

int main() {
  const size_t rows = (size_t)1 << 25;             // 2 GiB of 64-byte points
  const size_t n = 31457320;                       // entries of one 2^21-point fixed-base MSM
  Pt* table;
  uint32_t *idx, *out;
  CK(hipMalloc(&table, rows * sizeof(Pt)));
  CK(hipMalloc(&idx, n * 4));
  CK(hipMalloc(&out, ((size_t)1 << 24) * 4));
  CK(hipMemset(table, 0x5a, rows * sizeof(Pt)));
  fill_idx<<<(n + 255) / 256, 256>>>(idx, n, (uint32_t)rows, 12345);
  CK(hipDeviceSynchronize());
  const size_t threads = (n + kChunk - 1) / kChunk;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; rep++) {
    float ms[3];
    CK(hipEventRecord(e0));
    gather64<<<(threads + 255) / 256, 256>>>(table, idx, n, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms[0], e0, e1));
    CK(hipEventRecord(e0));
    idx_only<<<(threads + 255) / 256, 256>>>(idx, n, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms[1], e0, e1));
    CK(hipEventRecord(e0));
    stream16<<<8192, 256>>>((const uint4*)table, rows * sizeof(Pt) / 16, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms[2], e0, e1));
    printf("rep %d: gather64 %.3f ms (%zu x 64 B = %.3f GB gathered + %.3f GB indices), idx_only %.3f ms, "
           "stream16 %.3f ms (%.3f GB, %.0f GB/s)\n",
           rep, ms[0], n, n * 64.0 / 1e9, n * 4.0 / 1e9, ms[1], ms[2], rows * 64.0 / 1e9,
           rows * 64.0 / 1e9 / (ms[2] / 1e3));
  }
  CK(hipFree(table));
  CK(hipFree(idx));
  CK(hipFree(out));
  return 0;
}
