// Per-device compute engine: stream, NTT twiddles and MSM scratch.
#pragma once
#include "msm.h"
#include "ntt.h"

namespace nzcb {

struct Engine {
  int device = 0;
  hipStream_t stream = nullptr;
  NttTables ntt_tables;
  MsmScratch msm_scratch;
  Engine(int device, int max_log_ntt, size_t max_msm_points);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;
};

}  // namespace nzcb
