// Shared host-side helpers for the nzcb HIP library.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

#include "../../include/nzcb_internal.h"
#include "field.h"

namespace nzcb {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// Error codes: NZCB_* from include/nzcb.h. Fills `err` (may be NULL); capi_engine.hip.
void set_err(nzcb_err* err, int code, const char* msg);

// Kernel stores into pinned host memory (the prover's mailbox, the fixed-base MSM's window
// sums; round 6): plain stores, then a system-scope fence before the wave ends, so the host
// sees them once it has seen the kernel complete. Round 6 also tried one system-scope atomic
// store per 32-bit word and a wait for them (no L2 writeback): same box, 5-lane bench, three
// runs each, that cost 0.8 % of proofs/s against this (profiles/r6_sets_ab.txt, r6l: 36 uncached
// word writes per 144-byte window slot instead of nine 16-byte ones).
template <class T>
__device__ __forceinline__ void host_put(T* dst, const T& v) {
  *dst = v;
}
__device__ __forceinline__ void host_put_done() { __threadfence_system(); }


#define NZ_HIP(call)                                                                  \
  do {                                                                                \
    hipError_t e_ = (call);                                                           \
    if (e_ != hipSuccess)                                                             \
      throw ::nzcb::Error(NZCB_ERR_HIP, std::string("HIP error ") +           \
                                                    hipGetErrorString(e_) + " at " +  \
                                                    __FILE__ + ":" + std::to_string(__LINE__)); \
  } while (0)

// Guard words past the end of device buffers (the round-4 overrun of the
// three-coset quotient buffer surfaced as an illegal access two kernels later). While a
// GuardScope is alive on the calling thread (the prover's lane and proving-key
// allocations), every DevBuf::alloc adds kGuardBytes of kGuardByte past the end and
// registers them; guard_check() reads every registered guard back (capi_engine.hip).
constexpr size_t kGuardBytes = 4096;
constexpr unsigned char kGuardByte = 0xA5;
extern thread_local int g_guard_scope;
struct GuardScope {
  GuardScope() { g_guard_scope++; }
  ~GuardScope() { g_guard_scope--; }
  GuardScope(const GuardScope&) = delete;
  GuardScope& operator=(const GuardScope&) = delete;
};
void guard_register(void* base, size_t bytes);  // writes the pattern (synchronously)
void guard_unregister(void* base);
// every registered guard on `device` (-1: all devices): the number found damaged; `report`
// lists them (address, buffer bytes, first damaged offset)
int guard_check(int device, size_t* checked, std::string* report);

// Plain owning device buffer.
template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  bool owned = true;  // false: a view of another buffer (shared proving-key data)
  bool guarded = false;
  DevBuf() = default;
  explicit DevBuf(size_t count) { alloc(count); }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), n(o.n), owned(o.owned), guarded(o.guarded) {
    o.p = nullptr;
    o.n = 0;
    o.guarded = false;
  }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) {
      release();
      p = o.p; n = o.n; owned = o.owned; guarded = o.guarded;
      o.p = nullptr; o.n = 0; o.guarded = false;
    }
    return *this;
  }
  ~DevBuf() { release(); }
  void alloc(size_t count) {
    release();
    if (g_guard_scope > 0) {
      NZ_HIP(hipMalloc(&p, count * sizeof(T) + kGuardBytes));
      guard_register(p, count * sizeof(T));
      guarded = true;
    } else if (count) {
      NZ_HIP(hipMalloc(&p, count * sizeof(T)));
    }
    n = count;
    owned = true;
  }
  void alias(const DevBuf& o) {
    release();
    p = o.p;
    n = o.n;
    owned = false;
  }
  void release() {
    if (p && owned) {
      if (guarded) guard_unregister(p);
      (void)hipFree(p);
    }
    p = nullptr;
    n = 0;
    guarded = false;
  }
  size_t bytes() const { return n * sizeof(T); }
};

inline unsigned grid_for(size_t work, unsigned block, unsigned cap = 65535u * 16u) {
  size_t g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

inline int ilog2(uint64_t n) {
  int k = 0;
  while ((1ull << k) < n) k++;
  return k;
}

}  // namespace nzcb
