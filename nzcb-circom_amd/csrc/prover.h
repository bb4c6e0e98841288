// Device-resident PLONK prover (snarkjs 0.4.12 plonk_prove restated for gfx950).
#pragma once
#include <chrono>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "engine.h"
#include "zkey.h"

namespace nzcb {

struct AddRec {  // one addition, reordered by dependency level
  uint32_t ai, bi, dst, pad;
  Fr ac, bc;
};

// one proof's MSMs split by point range over several devices
// of this process. A shard holds the shifted-base tables of its PTau range and of its
// Lagrange-basis range (A, B, C) and per-slot MSM scratch; the scalar slice arrives by a
// device-to-device copy over xGMI and the 96-byte partial comes back to the host, where the
// partials are added.
struct MsmShard {
  static constexpr int kSlots = 3;
  int device = 0;
  size_t lo = 0, hi = 0;    // PTau points
  size_t llo = 0, lhi = 0;  // Lagrange-basis points (lhi = 0: none, the context commits A, B, C from coefficients)
  MsmBaseTable table, ltable;
  std::unique_ptr<MsmScratch> sc[kSlots];
  DevBuf<Fr> scal[kSlots];
  hipStream_t st[kSlots] = {nullptr, nullptr, nullptr};
  ~MsmShard();
};

struct Prover {
  // zkey facts
  uint32_t n = 0, n4 = 0, nVars = 0, nPublic = 0, nAdditions = 0, nConstraints = 0, nWit = 0;
  int power = 0;
  Fr k1, k2, wn, w2;
  std::vector<uint32_t> add_level_start;  // offsets into d_adds per level
  bool transcript_public = true;
  std::function<void(const std::string&)> log;

  std::unique_ptr<Engine> eng;
  // commitment pipeline: one MSM scratch + stream per concurrently running commitment
  static constexpr int kSlots = 3;
  std::unique_ptr<MsmScratch> msc[kSlots];
  hipStream_t aux[kSlots] = {nullptr, nullptr, nullptr};
  hipEvent_t ready[kSlots] = {nullptr, nullptr, nullptr};
  bool slot_split[kSlots] = {false, false, false};  // slot's MSM went to the other ranks (commit_finish gathers)
  bool slot_lag[kSlots] = {false, false, false};    // slot's MSM is over the Lagrange basis
  // round 1's interpolations of A, B, C (and the gate check) run on aux[2], overlapping
  // round 2; round 3 waits for side_done. pows_done: round 4's divPol1 tile powers (aux[2])
  hipEvent_t side_ready = nullptr, side_done = nullptr, pows_done = nullptr;
  ~Prover();
  // resident zkey data (LEM, as in the file)
  DevBuf<G1Affine> ptau;
  MsmBaseTable ptab;  // shifted PTau bases for the fixed-base MSM schedule
  // Lagrange-basis SRS (csrc/lagrange.hip): [L_k(tau)] (k < n), [tau^n] - [1],
  // [tau^(n+1)] - [tau], and its shifted-base table: A, B, C are committed from their
  // evaluations (mostly small scalars) instead of their coefficients
  DevBuf<G1Affine> ltau;
  MsmBaseTable ltab;
  bool lcommit = false;
  DevBuf<Fr> qm, ql, qr, qo, qc;  // [n coefs | 4n evals]
  DevBuf<Fr> sigma;               // 3 x [n | 4n]
  DevBuf<Fr> sig_h;               // 3 x n: sigma_k(w^i), contiguous (round 2)
  DevBuf<Fr> q_h;                 // 5 x n: qm..qc(w^i), contiguous (the gate check on H, quot3)
  DevBuf<Fr> w_h;                 // n: w^i (round 2's grand product)
  DevBuf<Fr> lagrange;            // nLagrange x [n | 4n]
  DevBuf<uint32_t> amap, bmap, cmap;
  DevBuf<AddRec> adds;
  DevBuf<Fr> root_lo, root_hi;    // w4^j, w4^(4096 k)
  DevBuf<Fr> x_lo;                // g * w4^j (coset points, with root_hi)
  DevBuf<Fr> g_lo, g_hi, gi_lo, gi_hi;  // g^j, g^-j split tables
  DevBuf<F29> g29, gi29;                 // g^j (j < n + 8) and g^-j / 4n (j < 4n), mul_fr29 operands
  Fr zh_inv[4];
  DevBuf<Fr> cq, cs, cl;          // coset evaluations: Qm..Qc (5 x 4n), sigma1..3 (3 x 4n), L_j (nl x 4n)
  // Three-coset quotient (quot3): the quotient is evaluated on cosets c_j H, c_j = g w4^j,
  // j < 3 (3n points, coset-major [j][m]) and t's top six coefficients come from the top
  // coefficients of A, B, C, Z and sigma (prove(), round 3)
  bool quot3 = false;
  DevBuf<Fr> cq3, cs3, cl3;       // Qm..Qc (5 x 3n), sigma1..3 (3 x 3n), L_j (nl x 3n)
  DevBuf<F29> tw3, itw3;          // c_j^k and c_j^-k / 4n (3 x n each), mul_fr29 operands
  Fr d3[3];                       // c_j^n = g^n w4^(j n)
  Fr sig_top[3][4];               // sigma_k coefficients n-4 .. n-1
  // per-proof working set
  DevBuf<Fr> wit;                 // nVars (witness + internal), Montgomery
  DevBuf<Fr> wtns_in;             // raw witness upload (normal form)
  DevBuf<Fr> A, B, C, Z;          // n (A, B, C: n + 2, the blinding scalars b_lo, b_hi at n, n + 1)
  DevBuf<Fr> pol_a, pol_b, pol_c, pol_z;  // n+2 / n+3
  DevBuf<Fr> A4, B4, C4, Z4, T, Tz, t;  // 4n (A4..Z4: coset evaluations)
  DevBuf<Fr> pol_r, pol_wxi, pol_wxiw;    // n+3, n+6, n+3
  DevBuf<Fr> blind;               // 12 (index 0 unused)
  DevBuf<Fr> scan_tmp;            // tile totals / heads of the round-2 and round-5 scans, and their levels
  DevBuf<Fr> lin_tab;             // 2 x LinTab (prover.hip) + tile powers: divPol1's tables for xi, xi w
  size_t lin_qn = 0;              // tile-power entries per table (n / kTileN + 3)
  Fr* lin_tile_pows(int k);       // Q then Qinv of slot k
  std::vector<Fr> lin_host;       // their host copies (Fr-sized words)
  DevBuf<Fr> eval_part;           // partial sums of polynomial evaluations
  DevBuf<F29> eval_pw;            // the evaluation points' powers x^t, t < 256
  DevBuf<uint32_t> flags;
  std::vector<Fr> host_part;  // (unused since round 6: the evaluations land in the mailbox)
  DevBuf<uint32_t> ntt_scr2;      // Z's transforms' inter-pass scratch (beside A, B, C's on aux[2])
  // The proof's mailbox (round 6): coherent pinned host memory that the
  // kernels producing the host's small per-proof inputs write directly, instead of one
  // hipMemcpyAsync (a blit dispatch that queued behind the other lanes' kernels) each:
  //   [0, 24) the top coefficients of A, B, C and Z (round 3's t recombination; k_tops)
  //   [24]    the check flags word (k_tops, k_div_check)
  //   [25, 27) prod num / prod den (round 2's copy check; k_perm_factors)
  //   [27, 27 + kEvalMax) evaluations (k_eval_sum)
  //   then A's nPublic public-gate values (the beta transcript) and witness[1..nPublic]
  //   (the public signals), both written by k_build_abc
  Fr* top_host = nullptr;
  static constexpr int kMbFlags = 24, kMbTotals = 25, kMbEvals = 27, kMbEvalMax = 8;
  size_t mb_apub = 0, mb_pubw = 0, mb_words = 0;

  int lane_id = 0;  // lane index on its device (the "lane k" trace mark of each proof)
  int fault = 0;  // nzcb_debug_inject_fault: NZCB_FAULT_* / NZCB_DEBUG_* for this lane's next proof
  // timings of the last proof (ms): [0..6] host wall clock of the whole proof and its
  // phases, [7] host time in the MSM calls (enqueue + waiting for results), [8] host time
  // enqueueing transforms, and with kernel statistics on (prof_gpu) the GPU time of [9] the
  // commitment MSMs and [10] the transforms: HIP event pairs around each one on its stream
  double tm[11] = {0};
  bool prof_gpu = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> span_ev;  // event pairs, created on first use
  std::vector<int> span_kind;                               // per pair in use: 0 MSM, 1 transform
  size_t spans_used = 0;
  size_t span_begin(int kind, hipStream_t s);
  void span_end(size_t i, hipStream_t s);
  void span_totals(double* msm_ms, double* ntt_ms);

  Prover(const uint8_t* zkey, size_t len, int device);
  Prover(const Prover& primary, int lane);  // extra lane sharing primary's proving key
  // Split every commitment MSM over devices[0] (this prover's device) and the others.
  void set_msm_devices(const std::vector<int>& devices);
  std::vector<std::unique_ptr<MsmShard>> shards;
  size_t own_hi = 0, own_lhi = 0;  // this device's PTau / Lagrange ranges are [0, own_hi) / [0, own_lhi) with shards
  // SURVEY.md §8e config 5 across processes (one rank per GPU, RCCL over xGMI): this
  // prover computes the PTau points [0, split_own) of every commitment and, when split_own_l
  // > 0, the Lagrange-basis points [0, split_own_l) of A, B and C; `split_send` hands the
  // commitment's scalars (HBM) to the other ranks as soon as they are ready (the slot with
  // NZCB_MSM_LAGRANGE for the Lagrange basis) and `split_gather` returns every rank's 64-byte
  // affine partial (rank order), which are added here. Both are caller callbacks (the
  // collectives live in the host runtime).
  nzcb_msm_send_fn split_send = nullptr;
  nzcb_msm_gather_fn split_gather = nullptr;
  void* split_user = nullptr;
  int split_world = 1;
  size_t split_own = 0, split_own_l = 0;
  void set_msm_split(int world, size_t own_points, size_t own_lagrange, nzcb_msm_send_fn send,
                     nzcb_msm_gather_fn gather, void* user);
  // witness: nWit x 32-byte LE normal-form values; blinding: 11 x 32-byte LE or null
  // witness_on_device: `witness` is a device pointer (HBM-resident input, no PCIe copy)
  void prove(const uint8_t* witness, size_t n_witness, const uint8_t* blinding, uint8_t* proof_out,
             uint8_t* pub_out, bool witness_on_device = false);

 private:
  hipStream_t st() const { return eng->stream; }
  void init_slots();
  void alloc_workspace();
  void to4t(const Fr* evals, Fr* coefs, Fr* evals4, const int* bidx, int nb, hipStream_t s = nullptr);
  void to4t_coefs(const Fr* evals, Fr* coefs, const int* bidx, int nb, hipStream_t s, uint32_t* scr = nullptr);
  void to4t_evals4(const Fr* coefs, Fr* evals4, int nb, hipStream_t s, uint32_t* scr = nullptr);
  void round3_quot3(const Fr& beta, const Fr& gamma, const Fr& alpha, hipStream_t s);
  void launch_gate_check(hipStream_t s);
  void copy_tops(hipStream_t s);  // the tops and flags into top_host; throws on a gate failure
  void commit_start(int slot, const Fr* scalars, size_t len, const MsmBaseTable* tab = nullptr,
                    const G1Affine* bases = nullptr, bool on_main = false);
  G1Affine commit_finish(int slot);
  void commit_start_abc(size_t len);  // A, B, C in one schedule (msm_enqueue_sets), main stream
  void commit_finish_abc(G1Affine& a, G1Affine& b, G1Affine& c);
  // np <= 8 evaluations p_j(x_j) (two launches, one host round trip)
  void eval_many(int np, const Fr* const* polys, const size_t* lens, const Fr* xs, Fr* out,
                 const std::function<void()>& overlap = nullptr);
  // y_i = x_i + d y_(i+1) with d from lin_tables slot `tab` (round 4 builds slots 0, 1 = xi, xi w)
  void div_pol1(const Fr* src, size_t m, int tab, const Fr& p0_adjust, Fr* dst, uint32_t flag_bit);
  void lin_tables(int k, const Fr& d, hipStream_t s);
  double ms_since(std::chrono::steady_clock::time_point t0);
  double msm_ms = 0, ntt_ms = 0;
};

}  // namespace nzcb
