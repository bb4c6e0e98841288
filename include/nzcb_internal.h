/*
 * nzcb internal ABI: kernel-level entry points for tests, microbenchmarks and tuning
 * (SURVEY.md §8d config 2). Exported by libnzcb.so next to the product ABI of nzcb.h, but
 * not part of the drop-in boundary and not stable.
 */
#ifndef NZCB_INTERNAL_H
#define NZCB_INTERNAL_H

#include "nzcb.h"

#ifdef __cplusplus
extern "C" {
#endif

/* HIP-event timing of the MSM bucket-accumulation kernel (the dominant kernel):
 * out = {total ms, launches, MSM points, bucket entries} accumulated since the last
 * reset; enable = 1 / 0 turns timing on / off and resets (waiting for the proofs in flight),
 * -1 only reads (without waiting: the totals may include a proof in flight). Timing adds no
 * host synchronisation (the entry count is copied with the MSM's window sums). */
int nzcb_ctx_kernel_stats(nzcb_ctx* ctx, int enable, double out[4]);

/* Guard words (csrc/common.h GuardScope): every device buffer a prover context allocates
 * (proving key, lanes' working sets, MSM and NTT scratch) carries 4 KiB of a known pattern
 * past its end. nzcb_debug_guard_check reads every guard on `device` (-1: all) back: 0
 * when all are intact, NZCB_ERR_INTERNAL with the damaged buffers in err otherwise
 * (checked / damaged: counts). Call it with no proof in flight. nzcb_debug_guard_selftest
 * writes one word past a fresh guarded buffer and checks that exactly that is found. */
int nzcb_debug_guard_check(int device, size_t* checked, int* damaged, nzcb_err* err);
int nzcb_debug_guard_selftest(int device, nzcb_err* err);

/* Fault injection (tests of the prover's own checks): the context's next proof, whichever
 * lane takes it, perturbs its quotient t after round 3 (kind NZCB_FAULT_QUOTIENT: t[1] += 1),
 * which the xi check must report as NZCB_ERR_INTERNAL "quotient check failed". One-shot per
 * context (until round 5 per lane: the lanes that did not take it stayed armed); kind 0
 * clears it. */
#define NZCB_FAULT_QUOTIENT 1
/* Not a fault: kind NZCB_DEBUG_GENERIC_K makes the next proof's grand product form
 * k1 beta w^i and k2 beta w^i by their own Shoup products (the path for k1, k2 other than
 * snarkjs' 2, 3) instead of 2 beta w^i and 3 beta w^i by additions; the proof must be the
 * same. One-shot per context, like the fault. */
#define NZCB_DEBUG_GENERIC_K 2
/* Kind NZCB_FAULT_LANE_ALLOC arms the context's next nzcb_ctx_set_lanes growth instead of a
 * proof: after its first new lane a real device allocation larger than HBM fails (HIP's
 * per-thread last error then holds the out-of-memory code, as after a real failed growth) and
 * the call returns NZCB_ERR_HIP. The rollback must leave lanes() at its old value, the
 * pool consistent and the thread's last error cleared. One-shot. */
#define NZCB_FAULT_LANE_ALLOC 3
int nzcb_debug_inject_fault(nzcb_ctx* ctx, int kind);

/* The 9x29-bit products of csrc/f29.h as compiled for the device (the generated column asm),
 * over `count` host items of 32-bit limb words (9 per value), for tests against exact
 * integers. op 1: mul_shoup(x, w, ws) (27 words in, 9 out); 2: mul_shoup_x2 (54 / 18);
 * 3: mul29<Fq29>(a, b) (18 / 9); 4: mul29x2<Fr29>(a, b, c, d) (36 / 18); 5: sqr29x2(a, c)
 * (18 / 18); 6: mul2sum29(a, b, c, d) (36 / 9). Synchronous; count <= 2^24. */
int nzcb_debug_f29(int device, int op, const uint32_t* in, size_t count, uint32_t* out, nzcb_err* err);

/* ---- Synthetic circuit + setup ------- */
/* Builds the seeded synthetic circuit of oracle/synth.py and its snarkjs-0.4
 * PLONK zkey with trapdoor tau (32-byte LE normal) on `device`. Buffers are
 * malloc'ed by the library; free them with nzcb_free. */
int nzcb_synth_setup(int power, int n_public, int n_inputs, uint64_t seed, uint32_t n_constraints,
                     const uint8_t* tau, int device, uint8_t** zkey_out, size_t* zkey_len, uint8_t** wtns_out,
                     size_t* wtns_len, nzcb_err* err);
/* Same with flags: NZCB_SYNTH_FREE_PUBLIC keeps the public signals off every gate but
 * their public-input gate, so any public values satisfy the circuit. The bench's
 * fullProve pipeline writes the nzcp outputs of each pass there (nzcb_nzcp_witness_dev). */
#define NZCB_SYNTH_FREE_PUBLIC 1u
int nzcb_synth_setup_ex(int power, int n_public, int n_inputs, uint64_t seed, uint32_t n_constraints, uint32_t flags,
                        const uint8_t* tau, int device, uint8_t** zkey_out, size_t* zkey_len, uint8_t** wtns_out,
                        size_t* wtns_len, nzcb_err* err);
/* ---- Kernel-level entry points ------------------------------------------------ */
typedef struct nzcb_engine nzcb_engine;
nzcb_engine* nzcb_engine_create(int device, int max_log_ntt, size_t max_msm_points, nzcb_err* err);
void nzcb_engine_destroy(nzcb_engine* e);
/* Host-buffer variants. Field elements are 32-byte LE Montgomery ("LEM", zkey layout). */
int nzcb_engine_ntt(nzcb_engine* e, const uint8_t* in_lem, uint8_t* out_lem, int log_n, int inverse, nzcb_err* err);
/* bases: n x 64-byte LEM affine; scalars: n x 32 B LE (Montgomery if scalars_mont);
 * out: 64-byte affine x||y LE normal (infinity = zeros). */
int nzcb_engine_msm(nzcb_engine* e, const uint8_t* bases_lem, const uint8_t* scalars, size_t n, int scalars_mont,
                    uint8_t* out_affine, nzcb_err* err);
/* Device-resident variants for benchmarks (pointers from nzcb_dev_alloc, nzcb.h). */
int nzcb_engine_ntt_dev(nzcb_engine* e, const void* in, void* out, int log_n, int inverse, nzcb_err* err);
int nzcb_engine_msm_dev(nzcb_engine* e, const void* bases, const void* scalars, size_t n, int scalars_mont,
                        uint8_t* out_affine, nzcb_err* err);
/* Average milliseconds per call of `reps` back-to-back device NTTs, timed with HIP
 * events on the engine's stream. */
int nzcb_engine_time_ntt(nzcb_engine* e, const void* in, void* out, int log_n, int inverse, int reps, double* ms,
                         nzcb_err* err);
/* Microbench inputs: n pseudo-random Fr (Montgomery, < 2^253)
 * from `seed`, and [s_i]G1 bases (LEM affine) from Montgomery scalars. Device pointers. */
int nzcb_engine_random_fr(nzcb_engine* e, void* dev_out, size_t n, uint64_t seed, nzcb_err* err);
int nzcb_engine_fixed_base(nzcb_engine* e, const void* dev_scalars_mont, size_t n, void* dev_out, nzcb_err* err);
/* Lagrange-basis SRS (csrc/lagrange.hip): dev_out[k] = [L_k(tau)] for k < 2^log_n, then
 * [tau^n] - [1] and [tau^(n+1)] - [tau], from ptau_n >= 2^log_n + 2 PTau points (LEM affine,
 * device pointers). The prover commits A, B, C from their evaluations with it. */
int nzcb_engine_lagrange_basis(nzcb_engine* e, const void* dev_ptau, size_t ptau_n, int log_n, void* dev_out,
                               nzcb_err* err);
/* Average wall ms per MSM over `reps` (host-synchronised) and the average bucket-
 * accumulation kernel ms (HIP events). */
int nzcb_engine_time_msm(nzcb_engine* e, const void* bases, const void* scalars, size_t n, int scalars_mont, int reps,
                         double* ms, double* acc_ms, nzcb_err* err);
/* Fixed-base schedule (the prover's): builds the shifted-base table of the first
 * n_table bases (the PTau tables' window, c = 20 by default: 2^(20w) multiples, 13 rows), then
 * runs the MSM of the first n. One-shot (table and scratch freed on return); for parity tests. */
int nzcb_engine_msm_fixed_dev(nzcb_engine* e, const void* bases, size_t n_table, const void* scalars, size_t n,
                              int scalars_mont, uint8_t* out_affine, nzcb_err* err);
/* The same with the table's window (16..20, 0 = the PTau tables' default) and schedule:
 * sparse = 1 is the Lagrange-basis table's (device-derived accumulation chunk, log-depth
 * carry trees; msm.hip dyn_chunk). */
int nzcb_engine_msm_table_dev(nzcb_engine* e, const void* bases, size_t n_table, const void* scalars, size_t n,
                              int scalars_mont, int window, int sparse, uint8_t* out_affine, nzcb_err* err);
/* `sets` (1..3) MSMs of n scalars each (device pointers scalars[0..sets)) over ONE Lagrange-window
 * table of the first n_table bases in one schedule (msm.hip msm_enqueue_sets: the prover's A, B,
 * C commitments since round 6); out_affine: sets x 64 bytes. */
int nzcb_engine_msm_sets_dev(nzcb_engine* e, const void* bases, size_t n_table, const void* const* scalars, int sets,
                             size_t n, int scalars_mont, uint8_t* out_affine, nzcb_err* err);
/* Per-phase MSM timing (HIP events, average over reps after three warm-up runs):
 * out[0] wall ms, out[1..7] keys, sort, offsets, accumulate, finalize, reduce, sums,
 * out[8] table build ms (fixed_base only), out[9] bucket entries per MSM (nonzero digits),
 * out[10] host ms per MSM from the device results' arrival to the affine result (the
 * window combination on the CPU: the Horner over the window slots), out[11] host ms of the
 * enqueue (kernel launches), out[12] of which the library radix sort's host call (generic
 * schedule). out holds 13 doubles. fixed_base: 0 generic, 1 the PTau tables' schedule, 2 the
 * Lagrange table's (window 17, sparse), 3 window 17 with the dense schedule. */
int nzcb_engine_time_msm2(nzcb_engine* e, const void* bases, const void* scalars, size_t n, int scalars_mont,
                          int fixed_base, int reps, double* out, nzcb_err* err);
/* Field self-test helpers: out[i] = a[i] * b[i] (Montgomery, device), n elements. */
int nzcb_engine_fr_mul(nzcb_engine* e, const uint8_t* a_lem, const uint8_t* b_lem, uint8_t* out_lem, size_t n,
                       int field_q, nzcb_err* err);

#ifdef __cplusplus
}
#endif
#endif
