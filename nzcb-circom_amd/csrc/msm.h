// BN254 G1 Pippenger MSM (expTau = G1.multiExpAffine).
#pragma once
#include <vector>

#include "common.h"
#include "ec.h"

namespace nzcb {

struct MsmScratch {
  size_t max_points = 0;
  DevBuf<uint32_t> offsets;   // first sorted position of each (window, bucket) key, + total at the end
  DevBuf<uint32_t> sorted;    // point index | sign << 31, grouped by bucket
  DevBuf<uint32_t> keys_in, keys_out, vals_in;
  DevBuf<uint8_t> sort_tmp;
  size_t sort_tmp_bytes = 0;
  DevBuf<G1xyzz> buckets;     // buckets whose entries lie in one accumulation chunk
  DevBuf<G1xyzz> carry_own;   // per chunk: partial sum of a bucket that starts in the chunk and spills over
  DevBuf<G1xyzz> carry_cont;  // per chunk: partial sum of a bucket that began in an earlier chunk
  DevBuf<G1xyzz> seg_tot;     // per (window, segment): sum_j (j+1) * bucket_j
  DevBuf<G1xyzz> seg_run;     // per (window, segment): sum_j bucket_j
  DevBuf<G1xyzz> win;         // per (window, sum slot): see msm_window_sums_kernel
  G1xyzz* host_win = nullptr;  // pinned
  size_t host_win_cap = 0;
  // shape of the MSM in flight (set by msm_enqueue, used by msm_finish)
  int cur_c = 0, cur_nw = 0, cur_nbits = 0, cur_seglen = 0;
  size_t cur_n = 0;
  uint32_t cur_nkeys = 0;
  // optional HIP-event timing of the bucket-accumulation kernel (bench.py roofline)
  bool prof = false;
  double prof_ms = 0;
  uint64_t prof_launches = 0, prof_points = 0, prof_entries = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  void init(size_t max_points);
  ~MsmScratch();
};

// Window size used for an MSM of n points.
int msm_window_bits(size_t n);

// Enqueue the whole MSM sum_i s_i * B_i on `st` (no host sync); msm_finish waits for
// it and folds the per-window sums on the host. bases: zkey PTau layout (LEM affine).
// scalars: Fr, Montgomery form if scalars_mont.
void msm_enqueue(MsmScratch& sc, const G1Affine* bases, const Fr* scalars, size_t n, bool scalars_mont,
                 hipStream_t st);
G1xyzz msm_finish(MsmScratch& sc, hipStream_t st);

inline G1xyzz msm(MsmScratch& sc, const G1Affine* bases, const Fr* scalars, size_t n, bool mont, hipStream_t st) {
  msm_enqueue(sc, bases, scalars, n, mont, st);
  return msm_finish(sc, st);
}

// Host helpers.
G1Affine xyzz_to_affine(const G1xyzz& p);

}  // namespace nzcb
