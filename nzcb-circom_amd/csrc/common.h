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


#define NZ_HIP(call)                                                                  \
  do {                                                                                \
    hipError_t e_ = (call);                                                           \
    if (e_ != hipSuccess)                                                             \
      throw ::nzcb::Error(NZCB_ERR_HIP, std::string("HIP error ") +           \
                                                    hipGetErrorString(e_) + " at " +  \
                                                    __FILE__ + ":" + std::to_string(__LINE__)); \
  } while (0)

// Plain owning device buffer.
template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  bool owned = true;  // false: a view of another buffer (shared proving-key data)
  DevBuf() = default;
  explicit DevBuf(size_t count) { alloc(count); }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), n(o.n), owned(o.owned) { o.p = nullptr; o.n = 0; }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) { release(); p = o.p; n = o.n; owned = o.owned; o.p = nullptr; o.n = 0; }
    return *this;
  }
  ~DevBuf() { release(); }
  void alloc(size_t count) {
    release();
    if (count) NZ_HIP(hipMalloc(&p, count * sizeof(T)));
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
    if (p && owned) (void)hipFree(p);
    p = nullptr;
    n = 0;
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
