// BN254 G1 Pippenger MSM (expTau = G1.multiExpAffine).
#pragma once
#include "common.h"
#include "ec.h"

namespace nzcb {

struct MsmScratch {
  size_t max_points = 0;
  DevBuf<uint32_t> counts;    // per (window, bucket) entry counts
  DevBuf<uint32_t> offsets;   // exclusive scan of counts, + total at the end
  DevBuf<uint32_t> cursor;    // scatter cursors
  DevBuf<uint32_t> sorted;    // point index | sign << 31, grouped by bucket
  DevBuf<G1xyzz> buckets;
  DevBuf<G1xyzz> carry_own;   // per chunk: partial sum of a bucket that starts in the chunk and spills over
  DevBuf<G1xyzz> carry_cont;  // per chunk: partial sum of a bucket that began in an earlier chunk
  DevBuf<uint32_t> own_key;
  DevBuf<G1xyzz> seg;         // per (window, segment) weighted partial sums
  DevBuf<G1xyzz> win;         // per-window sums
  DevBuf<uint8_t> scan_tmp;
  size_t scan_tmp_bytes = 0;
  // radix-sort bucketing (default; NZCB_MSM_SORT=atomic selects the histogram+scatter path)
  bool use_radix = true;
  DevBuf<uint32_t> keys_in, keys_out, vals_in;
  DevBuf<uint8_t> sort_tmp;
  size_t sort_tmp_bytes = 0;
  std::vector<G1xyzz> host_win;
  // optional HIP-event timing of the bucket-accumulation kernel (bench.py roofline)
  bool prof = false;
  double prof_ms = 0;
  uint64_t prof_launches = 0, prof_points = 0, prof_entries = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  void init(size_t max_points);
};

// Window size used for an MSM of n points.
int msm_window_bits(size_t n);

// Enqueue the MSM sum_i s_i * B_i on `st` and return the result after a stream sync.
// bases: zkey PTau layout (LEM affine). scalars: Fr, Montgomery form if scalars_mont.
G1xyzz msm(MsmScratch& sc, const G1Affine* bases, const Fr* scalars, size_t n, bool scalars_mont, hipStream_t st);

// Host helpers.
G1Affine xyzz_to_affine(const G1xyzz& p);

}  // namespace nzcb
