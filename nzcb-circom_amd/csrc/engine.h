// Per-device compute engine: stream, NTT twiddles and MSM scratch.
#pragma once
#include "msm.h"
#include "ntt.h"

namespace nzcb {

// [s_i] G1 (LEM affine) for Montgomery scalars, one thread per point (synth.hip).
void launch_fixed_base(const Fr* scalars_mont, size_t n, G1Affine* out, hipStream_t st);

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
