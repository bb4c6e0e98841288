/*
 * nzcb — MI355X-native PLONK prover for the nzcb circom circuit (C-ABI).
 *
 * This is the drop-in boundary under the reference's prover call:
 *   snarkjs.plonk.prove(zkeyFileName, witnessFileName, logger)      [EXT] snarkjs 0.4.12
 *   snarkjs.plonk.fullProve(input, wasmFile, zkeyFileName, logger)  [EXT]
 * pinned at /root/reference/package.json:18 and /root/reference/yarn.lock:7279-7292,
 * whose keys are produced at /root/reference/Makefile:54-62.
 * The N-API addon in nzcb-circom_amd/js/ binds these functions one-to-one
 * (see INTEGRATION.md). Plain pointers and sizes only; the caller owns every
 * buffer; nothing is retained after a call returns.
 *
 * Byte layouts
 *   zkey / wtns : snarkjs 0.4 binary files, unchanged.
 *   proof       : NZCB_PROOF_BYTES = 9 G1 affine points (A,B,C,Z,T1,T2,T3,Wxi,Wxiw),
 *                 each x||y as 32-byte little-endian normal-form integers
 *                 (infinity = 64 zero bytes), then 7 Fr evaluations
 *                 (eval_a,eval_b,eval_c,eval_s1,eval_s2,eval_zw,eval_r), 32 B LE each.
 *   public      : nPublic x 32-byte LE Fr (= witness[1..nPublic]).
 *   blinding    : 11 x 32-byte LE Fr (b1..b11), or NULL = drawn uniformly from the
 *                 OS CSPRNG per proof, as snarkjs's Fr.random() (zero-knowledge).
 *                 Fixed bytes (352 zero bytes included) give reproducible,
 *                 bit-exact proofs for tests; zero blinding is NOT zero-knowledge.
 *
 * This header is the product ABI. Kernel-level entry points for tests,
 * microbenchmarks and tuning (nzcb_engine_*, the synthetic-circuit setup, kernel timing)
 * are in nzcb_internal.h: they are exported by the same library but are not part of the
 * drop-in boundary and may change between releases. Until round 3 they were declared here;
 * code that used them through this header compiles with -DNZCB_WITH_INTERNAL (this header
 * then includes nzcb_internal.h) or includes nzcb_internal.h itself.
 */
#ifndef NZCB_H
#define NZCB_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NZCB_PROOF_BYTES (9 * 64 + 7 * 32)
#define NZCB_BLINDING_BYTES (11 * 32)

/* Error codes; messages reproduce the snarkjs 0.4.12 exception text. */
enum {
  NZCB_OK = 0,
  NZCB_ERR_ARG = 1,
  NZCB_ERR_FORMAT = 2,
  NZCB_ERR_NOT_PLONK = 3,     /* "zkey file is not plonk" */
  NZCB_ERR_CURVE = 4,         /* "Curve of the witness does not match the curve of the proving key" */
  NZCB_ERR_WITNESS_LEN = 5,   /* "Invalid witness length. Circuit: ..., witness: ..., ..." */
  NZCB_ERR_COPY = 6,          /* "Copy constraints does not match" */
  NZCB_ERR_T_DIV = 7,         /* "T Polynomial is not divisible" */
  NZCB_ERR_TZ = 8,            /* "Tz Polynomial is not well calculated" */
  NZCB_ERR_DIVPOL = 9,        /* "Polinomial does not divide" */
  NZCB_ERR_HIP = 10,
  NZCB_ERR_INTERNAL = 11
};

typedef struct nzcb_err {
  int code;
  char msg[256];
} nzcb_err;

typedef struct nzcb_ctx nzcb_ctx;
typedef void (*nzcb_log_fn)(void* user, const char* msg);

/* Library identity / devices. */
const char* nzcb_version(void);
int nzcb_device_count(void);

/* ---- Prover (replaces snarkjs plonk_prove) ---------- */

/* Parse a snarkjs 0.4 PLONK zkey and upload it to `device` (HBM-resident,
 * context-owned). Replaces the zkey read in snarkjs plonk_prove.js [EXT]. */
nzcb_ctx* nzcb_ctx_create(const uint8_t* zkey, size_t zkey_len, int device, nzcb_err* err);
/* SURVEY.md §8b's form: one context over a device set. Every device holds its own
 * HBM-resident copy of the proving key; nzcb_prove_batch spreads its items over the
 * lanes of all devices (nzcb_ctx_set_lanes sets lanes per device); single proofs run on
 * devices[0]. nzcb_ctx_create(z, len, d, err) is this with devices = {d}. */
nzcb_ctx* nzcb_ctx_create_devices(const uint8_t* zkey, size_t zkey_len, const int* devices, int ndev, nzcb_err* err);
/* The same from a zkey file (memory-mapped, nothing retained after the call): zkeys of
 * nzcp_live size (~3.9 GB) exceed what a Node.js Buffer holds. devices NULL = device 0. */
nzcb_ctx* nzcb_ctx_create_file(const char* zkey_path, const int* devices, int ndev, nzcb_err* err);
int nzcb_ctx_devices(const nzcb_ctx* ctx);
void nzcb_ctx_destroy(nzcb_ctx* ctx);

/* Optional progress logger (snarkjs `logger.debug` lines). */
void nzcb_ctx_set_logger(nzcb_ctx* ctx, nzcb_log_fn fn, void* user);

/* Include the public inputs in the beta transcript (1, default)
 * or hash A||B||C only (0). */
void nzcb_ctx_set_transcript_public(nzcb_ctx* ctx, int on);

/* Context facts: domain size, nPublic, nVars, nAdditions, nConstraints. */
int nzcb_ctx_info(const nzcb_ctx* ctx, uint32_t out[5]);

/* One proof. wtns = snarkjs .wtns bytes. proof_out: NZCB_PROOF_BYTES.
 * pub_out: pub_cap >= 32 * nPublic bytes. Returns NZCB_OK or an error code. */
int nzcb_prove(nzcb_ctx* ctx, const uint8_t* wtns, size_t wtns_len, const uint8_t* blinding, uint8_t* proof_out,
               uint8_t* pub_out, size_t pub_cap, nzcb_err* err);

/* Same with the witness given as nWitness x 32-byte LE field elements (no file header). */
int nzcb_prove_witness(nzcb_ctx* ctx, const uint8_t* witness, size_t n_witness, const uint8_t* blinding,
                       uint8_t* proof_out, uint8_t* pub_out, size_t pub_cap, nzcb_err* err);

/* Same with the witness already resident in HBM: dev_witness is a device pointer
 * (nzcb_dev_alloc) holding nWitness x 32-byte LE normal-form values. */
int nzcb_prove_device(nzcb_ctx* ctx, const void* dev_witness, size_t n_witness, const uint8_t* blinding,
                      uint8_t* proof_out, uint8_t* pub_out, size_t pub_cap, nzcb_err* err);

/* One proof with its own logger (NULL: the context's, nzcb_ctx_set_logger), the witness in
 * any of the three forms above: NZCB_WITNESS_WTNS (.wtns bytes, n = byte length),
 * NZCB_WITNESS_HOST (n x 32-byte LE values in host memory), NZCB_WITNESS_DEVICE (the same
 * in HBM). Concurrent calls on one context (several host threads; the N-API addon's
 * in-flight promises) each take a free lane and run at the same time; a call waits while
 * every lane is proving. nzcb_prove, nzcb_prove_witness and nzcb_prove_device are this
 * with the context's logger. */
#define NZCB_WITNESS_WTNS 0
#define NZCB_WITNESS_HOST 1
#define NZCB_WITNESS_DEVICE 2
int nzcb_prove_logged(nzcb_ctx* ctx, const void* witness, size_t n, int kind, const uint8_t* blinding,
                      uint8_t* proof_out, uint8_t* pub_out, size_t pub_cap, nzcb_log_fn log, void* log_user,
                      nzcb_err* err);

/* Proof lanes (default 1): each extra lane is a per-proof working set + streams on
 * the context's device (~6.5 GB at n = 2^21) sharing the HBM-resident proving key,
 * so nzcb_prove_batch keeps `lanes` proofs in flight and one proof's latency-bound
 * phases (Fiat-Shamir host steps, bucket reductions) overlap another's compute. A change
 * of the count waits for the proofs in flight (it rebuilds the lane pool); setting the
 * count the context already has returns at once. */
int nzcb_ctx_set_lanes(nzcb_ctx* ctx, int lanes, nzcb_err* err);
int nzcb_ctx_lanes(const nzcb_ctx* ctx);

/* Single-proof mode across GPUs: every commitment MSM of lane 0
 * is split by point range over devices[0..ndev) (devices[0] = the context's device); each
 * other device holds the shifted-base tables of its PTau range and of its range of the n + 2
 * Lagrange-basis points (A, B, C's commitments, when the context commits them in that basis),
 * receives its scalar slice by a peer copy over xGMI and returns one partial, which the host
 * adds. ndev = 1 restores the single-device schedule. Results are bit-identical either way. */
int nzcb_ctx_set_msm_devices(nzcb_ctx* ctx, const int* devices, int ndev, nzcb_err* err);

/* The same split across processes, one rank per GPU (each rank's
 * slice of the scalars by RCCL scatter, one 64-byte partial per rank back by gather; the
 * collectives live in the host runtime, e.g. torch.distributed, see nzcb/msmsplit.py). The
 * context (rank 0) computes PTau points [0, own_points) of every commitment of lane 0 and,
 * when own_lagrange > 0, Lagrange-basis points [0, own_lagrange) of A, B and C's commitments
 * (own_lagrange = 0 keeps those three whole on this rank), and calls
 *   send(user, slot, dev_scalars, count): the commitment's `count` scalars (32-byte
 *       Montgomery Fr, HBM of the context's device) are ready; the other ranks take the
 *       points [own, count) of it; called when the commitment starts. `slot` carries
 *       NZCB_MSM_LAGRANGE when the commitment is over the Lagrange basis (the n + 2 points
 *       [L_k(tau)] for k < n, [tau^n] - [1], [tau^(n+1)] - [tau]; a serving rank's table of
 *       its range comes from nzcb_msm_table_create_lagrange) rather than PTau
 *   gather(user, slot, own_partial, partials_out): returns world x 64 bytes, every rank's
 *       partial sum (affine x || y, 32-byte LE normal form, infinity = zeros) in rank
 *       order (own_partial at index 0); called when the commitment is needed, with the
 *       same slot value as its send
 * Up to 3 commitments (slot & 0xff = 0..2) are in flight at once. A callback returning
 * non-zero fails the proof. world = 1 or NULL callbacks restore the local schedule. */
#define NZCB_MSM_LAGRANGE 0x100
typedef int (*nzcb_msm_send_fn)(void* user, int slot, const void* dev_scalars, size_t count);
typedef int (*nzcb_msm_gather_fn)(void* user, int slot, const uint8_t* own_partial, uint8_t* partials_out);
int nzcb_ctx_set_msm_split(nzcb_ctx* ctx, int world, size_t own_points, size_t own_lagrange,
                           nzcb_msm_send_fn send, nzcb_msm_gather_fn gather, void* user, nzcb_err* err);

/* `count` independent proofs over the context's lanes (SURVEY.md §8b nzcb_prove_batch,
 * §8e batch mode). witnesses[i]: nWitness x 32-byte LE normal-form values, host memory,
 * or device pointers when witness_on_device. blindings: count x NZCB_BLINDING_BYTES or
 * NULL (random per proof, see `blinding` above). proofs_out: count x NZCB_PROOF_BYTES. pubs_out: count x pub_stride
 * (pub_stride >= 32 * nPublic). Returns the error of the lowest failing index. */
int nzcb_prove_batch(nzcb_ctx* ctx, const void* const* witnesses, size_t n_witness, int count, int witness_on_device,
                     const uint8_t* blindings, uint8_t* proofs_out, uint8_t* pubs_out, size_t pub_stride,
                     nzcb_err* err);
/* As nzcb_prove_batch, but a failed proof does not stop the batch: every
 * item is proved, status_out[i] (count ints) receives 0 or proof i's error code, and a
 * failed item's proof and public bytes are zeroed. Returns (and reports in err) the
 * error of the lowest failing index, 0 when all succeed. */
int nzcb_prove_batch_status(nzcb_ctx* ctx, const void* const* witnesses, size_t n_witness, int count,
                            int witness_on_device, const uint8_t* blindings, uint8_t* proofs_out, uint8_t* pubs_out,
                            size_t pub_stride, int* status_out, nzcb_err* err);

/* Milliseconds of the last proof's phases. Host wall clock: [0] total [1] witness
 * upload+additions+ABC [2] round1 [3] round2 [4] round3 [5] round4 [6] round5, [7] host time
 * inside the MSM calls (enqueue + waiting for their results), [8] host time enqueueing the
 * transforms. GPU time (HIP events around each commitment MSM / each transform on its
 * stream, only while nzcb_ctx_kernel_stats is on, else -1): [9] MSMs [10] transforms.
 * Returns the number of values written (cap <= 11). */
int nzcb_ctx_last_timings(const nzcb_ctx* ctx, double* ms, int cap);

/* snarkjs-format JSON ({proof}, [publicSignals]) from the binary outputs. */
int nzcb_proof_to_json(const uint8_t* proof, char* out, size_t cap);
int nzcb_public_to_json(const uint8_t* pub, int n_public, char* out, size_t cap);

/* ---- Verification key, verifier, Solidity calldata ----
 * Host-only (no GPU needed). Binary verification key, NZCB_VK_BYTES:
 *   u32 nPublic | u32 power | k1, k2 (Fr, 32 B LE) | Qm Ql Qr Qo Qc S1 S2 S3 (G1 x||y,
 *   32 B LE each, infinity = zeros) | X_2 (x.c0 x.c1 y.c0 y.c1, 32 B LE) | w (Fr, 32 B LE)
 * Replaces snarkjs `zkey export verificationkey` (/root/reference/Makefile:56,61). */
#define NZCB_VK_BYTES (8 + 2 * 32 + 8 * 64 + 4 * 32 + 32)
int nzcb_vk_from_zkey(const uint8_t* zkey, size_t zkey_len, uint8_t* vk_out, nzcb_err* err);
/* The same from a zkey file, memory-mapped (zkeys past 2 GiB, e.g. nzcp_live's ~3.9 GB, which
 * `snarkjs zkey export verificationkey|solidityverifier nzcp_live_final.zkey` reads,
 * /root/reference/Makefile:61-62). */
int nzcb_vk_from_zkey_file(const char* zkey_path, uint8_t* vk_out, nzcb_err* err);
/* verification_key.json text (snarkjs layout); returns 0, or the needed size if cap is short. */
int nzcb_vk_to_json(const uint8_t* vk, char* out, size_t cap);
/* snarkjs plonk.verify: *valid = 1 if the proof (NZCB_PROOF_BYTES) is valid for the public
 * signals (n_public x 32 B LE), else 0. transcript_public as nzcb_ctx_set_transcript_public. */
int nzcb_verify(const uint8_t* vk, const uint8_t* proof, const uint8_t* pub, int n_public, int transcript_public,
                int* valid, nzcb_err* err);
/* snarkjs `zkey export soliditycalldata` for PLONK (/root/reference/Makefile:57,62 verifier):
 * "0x<proof hex>,[\"0x<pub>\",...]"; returns 0, or the needed size if cap is short. */
int nzcb_proof_to_calldata(const uint8_t* proof, const uint8_t* pub, int n_public, char* out, size_t cap);
/* snarkjs `zkey export solidityverifier` (/root/reference/Makefile:57,62; the contract
 * /root/reference/deploy-script.js:4-7 deploys): a Solidity PLONK verifier for this key,
 * verifyProof(bytes proof, uint256[] pubSignals) taking the soliditycalldata arguments
 * above. contract_name: NULL = "PlonkVerifier" (snarkjs's name; the reference's deploy
 * script asks for "Verifier"). transcript_public as nzcb_verify. Returns 0, the needed
 * size if cap is short, or -1 for a bad key or name. Parity unpinned (csrc/solidity.cpp). */
int nzcb_vk_to_solidity(const uint8_t* vk, const char* contract_name, int transcript_public, char* out, size_t cap);

/* ---- nzcp witness -----------------------------------
 * The semantic signals and public outputs of NZCPPubIdentity
 * (/root/reference/circuits/nzcptpl.circom:444-655, cbortpl.circom, quinSelector.circom)
 * for a batch of passes, one GPU workgroup per pass. Replaces, for the signals the
 * proof's public inputs depend on, circom_runtime's
 *   WitnessCalculator.calculateWitness(input, sanityCheck)   [EXT] circom_runtime 0.1.17
 * as called by snarkjs plonk.fullProve (wtns_calculate) and by the reference tests
 * (test/nzcp.js:42 `cir.calculateWitness(input, true)`).
 * Inputs per pass: the main's input signals in declaration order, each a 32-byte LE
 * field element (values >= r are reduced): toBeSigned[8*max_tbs_bytes] (bits, MSB
 * first per byte, test/helpers/utils.js:2-10), toBeSignedLen, data[160]
 * (nzcb_nzcp_input_signals() elements). Status codes mirror the circuit's failing
 * constraint or assert (the first one in template order); oracle/nzcp_circuit.py
 * is the CPU restatement with the same codes. */
enum {
  NZCB_NZCP_OK = 0,
  NZCB_NZCP_ERR_BIT = 1,        /* toBeSigned[i] * (toBeSigned[i] - 1) === 0 (detail = i) */
  NZCB_NZCP_ERR_LEN = 2,        /* toBeSignedLen < MaxToBeSignedBytes + 1 */
  NZCB_NZCP_ERR_RANGE = 3,      /* a LessThan / Num2Bits operand outside its bit range */
  NZCB_NZCP_ERR_SELECT = 4,     /* QuinSelector index >= choices (detail = index) */
  NZCB_NZCP_ERR_NOT_MAP = 5,    /* ReadMapLength: CBOR type is not a map */
  NZCB_NZCP_ERR_UINT23 = 6,     /* DecodeUint23: map length > 23 */
  NZCB_NZCP_ERR_NOT_STRING = 7, /* ReadStringLength: CBOR type is not a string */
  NZCB_NZCP_ERR_UNPINNED = 8    /* negative toBeSignedLen: Sha256Var behaviour not on disk */
};

/* NZCPPubIdentity(IsLive, MaxToBeSignedBytes, MaxCborArrayLenVC, MaxCborMapLenVC, ...):
 * nzcp_live = {1, 351, 0, 4}, nzcp_example = {0, 314, 0, 4} (circuits/nzcp_*.circom). */
typedef struct nzcb_nzcp_params {
  int32_t is_live;          /* CWT claims map at byte 30 (live) or 27 (example) */
  int32_t max_tbs_bytes;    /* 1..512 */
  int32_t max_array_len_vc; /* 0..8 */
  int32_t max_map_len_vc;   /* 0..32 */
} nzcb_nzcp_params;

/* One pass's result. On status != OK every other field except detail is zero. */
typedef struct nzcb_nzcp_record {
  int32_t status;
  int32_t detail;
  uint32_t exp;             /* CWT claim 4 */
  int32_t vc_pos;           /* FindCWTClaims.vcPos */
  int32_t given_len, family_len, dob_len, nullifier_len;
  uint8_t tbs_sha256[32];   /* SHA-256(ToBeSigned) */
  uint8_t nullifier_sha512[64];
  uint8_t nullifier[64];    /* "given,family,dob" zero-padded (ConstructNullifier.result) */
  uint8_t pub[3][32];       /* out[0..2] = witness[1..3], 32-byte LE normal-form Fr */
} nzcb_nzcp_record;

size_t nzcb_nzcp_input_signals(const nzcb_nzcp_params* prm);
/* Host buffers: inputs count x nzcb_nzcp_input_signals() x 32 B; records: count. */
int nzcb_nzcp_witness(int device, const nzcb_nzcp_params* prm, const uint8_t* inputs, int count,
                      nzcb_nzcp_record* records, nzcb_err* err);
/* Device buffers, asynchronous on `stream` (a hipStream_t, NULL = default stream).
 * dev_records may be NULL. When dev_witness is not NULL, pass i's out[0..2] are also
 * written as witness[1..3] of the witness at dev_witness + i * witness_stride (bytes),
 * so the prover's public inputs come straight from the pass (fullProve on device). */
int nzcb_nzcp_witness_dev(int device, const nzcb_nzcp_params* prm, const void* dev_inputs, int count,
                          void* dev_records, void* dev_witness, size_t witness_stride, void* stream,
                          nzcb_err* err);

/* ---- Witness programs: the circom witness calculator on the GPU ------------------
 * Replaces circom_runtime's calculateWitness / snarkjs wtns_calculate (circom_runtime
 * 0.1.17, /root/reference/yarn.lock:2496) for circuits
 * compiled by nzcb-circom_amd/nzcb/circuit.py (nzcp_live = NZCPPubIdentity(1, 351, 0, 4,
 * 2, 4), nzcb/nzcpgen.py). The program (format: csrc/wvm.hip) is uploaded once; each
 * run computes `count` full witnesses, one workgroup each.
 *   inputs : count x (n_pub_in + n_prv_in) x 32-byte LE field elements, the main's
 *            input signals in declaration order (as nzcb_nzcp_input_signals for nzcp)
 *   witness: witness i at dev_witness + i * witness_stride: n_wires x 32-byte LE normal
 *            form (wire 0 = 1, outputs, inputs, intermediate signals), the wtns order
 *            that nzcb_prove_device / nzcb_prove_batch take
 *   status : per witness, 0 or the failure code of the first failing check in circuit
 *            order (nzcp: NZCB_NZCP_* codes), as circom's calculator throws */
typedef struct nzcb_wprog nzcb_wprog;
nzcb_wprog* nzcb_wprog_create(const uint8_t* prog, size_t len, int device, nzcb_err* err);
void nzcb_wprog_destroy(nzcb_wprog* prog);
/* info: n_wires, n_outputs, n_pub_inputs, n_prv_inputs, n_levels */
int nzcb_wprog_info(const nzcb_wprog* prog, uint32_t info[5]);
/* Device buffers; stream may be NULL; returns after the statuses are on the host. */
int nzcb_wprog_run_dev(nzcb_wprog* prog, const void* dev_inputs, int count, void* dev_witness,
                       size_t witness_stride, int32_t* status_out, void* stream, nzcb_err* err);
/* Host buffers: witness_out receives count x n_wires x 32 bytes. */
int nzcb_wprog_run(nzcb_wprog* prog, const uint8_t* inputs, int count, uint8_t* witness_out,
                   int32_t* status_out, nzcb_err* err);
/* Re-index a witness program to another wire order by signal name (a zkey
 * built from circom's own r1cs, /root/reference/Makefile:12-15,59-62, expects circom's
 * wire order). own_sym: the program's .sym text (nzcb/circuit.py Circuit.write_sym);
 * target_sym: the .sym of the target order (e.g. circom's nzcp_live.sym; lines
 * "label,wire,component,name", wire -1 = optimized out). Target wire t gets the program
 * signal of the same name; wire 0 stays the constant 1. The result (malloc'ed, release
 * with nzcb_free) runs like any program and writes witnesses of the target's wire count.
 * Fails with NZCB_ERR_FORMAT, *unmatched = the count, when a target signal has no
 * counterpart. Parity of the names with circom's own .sym is unpinned (nzcb/nzcpgen.py). */
int nzcb_wprog_remap(const uint8_t* prog, size_t prog_len, const char* own_sym, size_t own_len,
                     const char* target_sym, size_t target_len, uint8_t** prog_out, size_t* prog_out_len,
                     uint32_t* unmatched, nzcb_err* err);

/* ---- Setup ------------------------------------------ */
/* snarkjs `plonk setup <r1cs> <ptau> <zkey>` (snarkjs 0.4.12 plonk_setup.js, run at
 * /root/reference/Makefile:55,60): iden3 r1cs + powers-of-tau file -> snarkjs-0.4 PLONK
 * zkey (malloc'ed, release with nzcb_free). Uses the ptau's tauG1 (section 2) and
 * tauG2 (section 3); NTTs and commitments run on `device`. */
int nzcb_plonk_setup(const uint8_t* r1cs, size_t r1cs_len, const uint8_t* ptau, size_t ptau_len, int device,
                     uint8_t** zkey_out, size_t* zkey_len, nzcb_err* err);
/* A powers-of-tau file (sections 1-3 of the snarkjs ptau layout: header, tauG1 =
 * [tau^i]G1 for i < 2^(power+1) - 1, tauG2 = [1]G2, [tau]G2) for a trapdoor tau (32 B LE),
 * built on `device`; malloc'ed, release with nzcb_free. The offline stand-in for
 * powersOfTau28_hez_final_21.ptau (/root/reference/README.md:40, Makefile:60). */
int nzcb_ptau_synth(int power, const uint8_t* tau, int device, uint8_t** ptau_out, size_t* ptau_len, nzcb_err* err);
void nzcb_free(void* p);

/* ---- HBM buffers (witnesses for nzcb_prove_device / nzcb_prove_batch on device) ---- */
void* nzcb_dev_alloc(size_t bytes);
/* The same on `device`; the calling thread's current device is left as it was (the N-API
 * addon's per-call threads allocate witness buffers on the witness program's device). */
void* nzcb_dev_alloc_on(int device, size_t bytes);
void nzcb_dev_free(void* p);
int nzcb_memcpy_h2d(void* dst, const void* src, size_t bytes);
int nzcb_memcpy_d2h(void* dst, const void* src, size_t bytes);
int nzcb_memcpy_d2d(void* dst, const void* src, size_t bytes);
/* The same ordered on a HIP stream (no host wait): work enqueued on `stream` afterwards
 * sees the copy (nzcb/msmsplit.py: scalars into the scatter rows on torch's stream). */
int nzcb_memcpy_d2d_async(void* dst, const void* src, size_t bytes, void* stream);

/* ---- Serving side of nzcb_ctx_set_msm_split (one per serving rank) ---------------- */
/* A resident fixed-base MSM table over n device bases (affine LEM, e.g. a PTau range),
 * the prover's shifted-base schedule for PTau (c = 20): the serving ranks of nzcb_ctx_set_msm_split
 * keep one and answer every commitment with one run. out_affine: 64 bytes, x || y normal
 * form LE (infinity = zeros); scalars: `count` <= n 32-byte values in HBM, Montgomery
 * form when scalars_mont (the prover's coefficients). */
typedef struct nzcb_msm_table nzcb_msm_table;
nzcb_msm_table* nzcb_msm_table_create(int device, const void* dev_bases, size_t n, nzcb_err* err);
/* The serving side of the Lagrange-basis commitments (NZCB_MSM_LAGRANGE): the points [lo, hi)
 * of the n + 2-point Lagrange basis of a 2^log_n domain ([L_k(tau)] for k < n, then
 * [tau^n] - [1], [tau^(n+1)] - [tau]), computed on `device` from its PTau (ptau_n >= n + 2
 * affine LEM points in HBM, e.g. a zkey's section 14) by the elliptic-curve inverse NTT the
 * prover runs at context creation, and kept as a table of the Lagrange window and its
 * schedule for small scalars. Scalars passed to nzcb_msm_table_run are the range's slice. */
nzcb_msm_table* nzcb_msm_table_create_lagrange(int device, const void* dev_ptau, size_t ptau_n, int log_n, size_t lo,
                                               size_t hi, nzcb_err* err);
int nzcb_msm_table_run(nzcb_msm_table* t, const void* dev_scalars, size_t count, int scalars_mont,
                       uint8_t* out_affine, nzcb_err* err);
void nzcb_msm_table_destroy(nzcb_msm_table* t);

#ifdef __cplusplus
}
#endif
#ifdef NZCB_WITH_INTERNAL  /* the pre-round-4 declarations (source compatibility) */
#include "nzcb_internal.h"
#endif
#endif
