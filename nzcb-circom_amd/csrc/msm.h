// BN254 G1 Pippenger MSM (expTau = G1.multiExpAffine).
#pragma once
#include <vector>

#include "common.h"
#include "ec.h"
#include "f29.h"

namespace nzcb {

// Precomputed shifted bases for fixed-base MSMs (the prover's PTau): row w holds
// 2^(c*w) * B_i (LEM affine), so every window's digits land in ONE bucket set and
// the per-window bucket reductions and the window Horner disappear.
struct MsmBaseTable {
  DevBuf<G1Affine> q;  // affine, coordinates x * 2^261 mod p (Montgomery-261, csrc/f29.h)
  size_t n = 0, stride = 0;
  int c = 0, nw = 0;
  // rows of 2^-256 B_i: the MSM then takes Montgomery-256 scalars as they are (mont = true
  // is required; msm.hip msm_table_kernel)
  bool mont_folded = false;
  // the sparse schedule (msm.hip dyn_chunk: device-derived chunk, log-depth carry trees) for
  // tables whose scalars are mostly small (the Lagrange basis: A, B, C's gate values); the
  // result is the same point either way
  bool sparse = false;
  void build(const G1Affine* bases, size_t n, int c, hipStream_t st, bool fold_mont = false);
};

// Window size of the table-based (fixed-base) MSM: 20 bits by default (13 table rows,
// 2^19 buckets; round 5); NZCB_FB_WINDOW = 16..20 overrides it.
int fixed_base_window();
// Window of the Lagrange-basis table (A, B, C commitments of small witness values: 17):
// their few entries do not pay for a larger bucket set.
int lagrange_window();
// the Lagrange tables' schedule (round 6): the sparse one (device-derived chunk, carry trees)
// with NZCB_SPARSE=1; off by default: on nzcp_live's A, B, C it cost 0.8-1.3 % of proofs/s
// against the dense schedule (profiles/r6_sets_ab.txt) for no single-proof latency gain
bool lagrange_sparse();

struct MsmScratch {
  size_t max_points = 0;
  int max_lsets = 1;  // Lagrange-table MSMs one schedule can take at once (msm_enqueue_sets)
  DevBuf<uint32_t> offsets;   // first sorted position of each bucket key, + total at the end
  DevBuf<uint32_t> sorted;    // base index | sign << 31, grouped by bucket
  DevBuf<uint32_t> keys_in, keys_out, vals_in;
  DevBuf<uint8_t> sort_tmp;
  size_t sort_tmp_bytes = 0;
  // fixed-base bucketing (msm.hip msm_bin_hist_kernel): per (high key byte, tile)
  // counts, scanned in place, and the values grouped by high byte
  DevBuf<uint32_t> bin_counts, vals_mid;
  DevBuf<uint32_t> lo_seg;    // per (bucket_lo work item, low index): count, then its first position
  DevBuf<G1xyzz> buckets;     // generic: buckets whose entries lie in one accumulation chunk
  DevBuf<G1xyzz> carry_own;   // per chunk: partial sum of a bucket that starts in the chunk and spills over
  DevBuf<G1xyzz> carry_cont;  // per chunk: partial sum of a bucket that began in an earlier chunk
  // fixed-base schedule: buckets and carries stay in radix 2^29 (Montgomery-261)
  DevBuf<Xyzz29> buckets29, carry_own29, carry_cont29;
  DevBuf<uint32_t> large;     // [count, bucket ids...] of buckets with long carry runs
  DevBuf<uint32_t> large_off;  // fixed base: piece offsets of the listed buckets (msm_large_scan_kernel)
  DevBuf<Xyzz29> large_part;   // fixed base: one partial sum per piece
  // fixed-base window sum (msm.hip msm_tile29_kernel): row / column partials per tile, lines
  DevBuf<Xyzz29> rowp29, colp29, lines29;
  DevBuf<G1xyzz> seg_tot;     // generic: per (bucket set, segment): sum_j (j+1) * bucket_j
  DevBuf<G1xyzz> seg_run;     // generic: per (bucket set, segment): sum_j bucket_j
  DevBuf<G1xyzz> parts;       // generic: per (set, sum slot, part): partial plain sums
  DevBuf<G1xyzz> win;         // per (set, sum slot): see msm_sums_kernel / msm_slots29_kernel
  G1xyzz* host_win = nullptr;  // pinned
  uint32_t* host_total = nullptr;  // pinned (after host_win's slots): the entry count (prof)
  size_t host_win_cap = 0;
  // shape of the MSM in flight (set by msm_enqueue, used by msm_finish)
  int cur_c = 0, cur_nsets = 0, cur_nbits = 0, cur_seglen = 0;
  bool cur_fixed = false, cur_sparse = false;
  int cur_a = 0, cur_hb = 0;  // fixed base: column / row bits of the window sum
  int cur_msets = 1;          // fixed base: MSMs in the schedule (msm_enqueue_sets)
  size_t cur_n = 0;
  uint32_t cur_nkeys = 0;
  // optional HIP-event timing: accumulation kernel (bench.py roofline) and, with
  // prof_phases, every phase (keys, sort, offsets, accumulate, finalize, reduce, sums)
  bool prof = false, prof_phases = false;
  double prof_ms = 0;
  double phase_ms[7] = {0, 0, 0, 0, 0, 0, 0};
  double host_ms = 0;          // msm_finish's CPU part (prof_phases)
  double enqueue_ms = 0;       // msm_enqueue's host time (prof_phases)
  double sort_host_ms = 0;     // of which the library radix sort's host call (generic schedule)
  uint64_t prof_launches = 0, prof_points = 0, prof_entries = 0;
  hipEvent_t ev[8] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  hipEvent_t done = nullptr;  // recorded after the window sums' copy to host_win (msm_finish waits on it)
  // lagrange_sets: size for msm_enqueue_sets of that many MSMs over a Lagrange-window table;
  // generic = false: table schedules only (no generic sort / 8x32 arrays)
  void init(size_t max_points, bool fixed_base = false, int lagrange_sets = 1, bool generic = true);
  ~MsmScratch();
};

// Window size of the generic (variable-base) MSM of n points.
int msm_window_bits(size_t n);

// Enqueue the whole MSM sum_i s_i * B_i on `st` (no host sync); msm_finish waits for
// it and folds the bucket-set sums on the host. bases: zkey PTau layout (LEM affine).
// scalars: Fr, Montgomery form if scalars_mont. With `table` (built from the same
// bases, n <= table->n) the fixed-base schedule is used.
void msm_enqueue(MsmScratch& sc, const G1Affine* bases, const Fr* scalars, size_t n, bool scalars_mont,
                 hipStream_t st, const MsmBaseTable* table = nullptr);
G1xyzz msm_finish(MsmScratch& sc, hipStream_t st);
// Several fixed-base MSMs over ONE table in one schedule (MsmScratch sized with lagrange_sets >=
// sets): one bucketing, accumulation and carry reduction over sets x 2^(c-1) buckets, window sums
// per set (round 6: A, B, C over the Lagrange basis). scalars[s]: n values each.
void msm_enqueue_sets(MsmScratch& sc, const Fr* const* scalars, int sets, size_t n, bool scalars_mont,
                      hipStream_t st, const MsmBaseTable* table);
void msm_finish_sets(MsmScratch& sc, hipStream_t st, G1xyzz* out);

inline G1xyzz msm(MsmScratch& sc, const G1Affine* bases, const Fr* scalars, size_t n, bool mont, hipStream_t st,
                  const MsmBaseTable* table = nullptr) {
  msm_enqueue(sc, bases, scalars, n, mont, st, table);
  return msm_finish(sc, st);
}

// Host helpers.
G1Affine xyzz_to_affine(const G1xyzz& p);

}  // namespace nzcb
