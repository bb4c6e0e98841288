"""ctypes binding of ``libnzcb.so`` (the C-ABI in ``include/nzcb.h``).

Host-side mirror of the reference's prover interface for this path
(snarkjs 0.4.12 ``plonk.prove(zkeyFileName, witnessFileName, logger)`` [EXT],
``/root/reference/package.json:18``): ``plonk.prove`` takes a
zkey and a witness (paths or bytes) and returns ``{proof, publicSignals}`` in
snarkjs's decimal-string JSON layout, raising with snarkjs's error text.

The library is the product: there is no CPU fallback. Loading fails loudly when
``lib/libnzcb.so`` has not been built, and every compute call needs a HIP device.
"""
from __future__ import annotations

import ctypes
import json
import os
from ctypes import POINTER, c_char, c_double, c_int, c_size_t, c_uint8, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NZCB_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libnzcb.so"))

PROOF_BYTES = 9 * 64 + 7 * 32
BLINDING_BYTES = 11 * 32
VK_BYTES = 8 + 2 * 32 + 8 * 64 + 4 * 32 + 32
PROOF_POINTS = ("A", "B", "C", "Z", "T1", "T2", "T3", "Wxi", "Wxiw")
PROOF_EVALS = ("eval_a", "eval_b", "eval_c", "eval_s1", "eval_s2", "eval_zw", "eval_r")
VK_POINTS = ("Qm", "Ql", "Qr", "Qo", "Qc", "S1", "S2", "S3")

ERROR_NAMES = {
    0: "OK", 1: "ARG", 2: "FORMAT", 3: "NOT_PLONK", 4: "CURVE", 5: "WITNESS_LEN", 6: "COPY",
    7: "T_DIV", 8: "TZ", 9: "DIVPOL", 10: "HIP", 11: "INTERNAL",
}

EXPORTED_SYMBOLS = [
    "nzcb_version", "nzcb_device_count", "nzcb_ctx_create", "nzcb_ctx_destroy", "nzcb_ctx_set_logger",
    "nzcb_ctx_set_transcript_public", "nzcb_ctx_info", "nzcb_prove", "nzcb_prove_witness", "nzcb_prove_device",
    "nzcb_ctx_kernel_stats",
    "nzcb_ctx_last_timings", "nzcb_proof_to_json", "nzcb_public_to_json", "nzcb_synth_setup", "nzcb_free",
    "nzcb_engine_create", "nzcb_engine_destroy", "nzcb_engine_ntt", "nzcb_engine_msm", "nzcb_dev_alloc",
    "nzcb_dev_free", "nzcb_memcpy_h2d", "nzcb_memcpy_d2h", "nzcb_engine_ntt_dev", "nzcb_engine_msm_dev",
    "nzcb_engine_time_ntt", "nzcb_engine_fr_mul", "nzcb_engine_random_fr", "nzcb_engine_fixed_base",
    "nzcb_engine_time_msm", "nzcb_engine_msm_fixed_dev", "nzcb_engine_msm_table_dev", "nzcb_engine_msm_sets_dev", "nzcb_engine_time_msm2", "nzcb_ctx_set_lanes",
    "nzcb_ctx_lanes", "nzcb_prove_batch", "nzcb_vk_from_zkey", "nzcb_vk_from_zkey_file", "nzcb_vk_to_json", "nzcb_verify",
    "nzcb_proof_to_calldata", "nzcb_vk_to_solidity", "nzcb_engine_lagrange_basis", "nzcb_ctx_set_msm_devices", "nzcb_nzcp_input_signals", "nzcb_nzcp_witness",
    "nzcb_nzcp_witness_dev", "nzcb_synth_setup_ex", "nzcb_memcpy_d2d",
    "nzcb_plonk_setup", "nzcb_prove_batch_status", "nzcb_wprog_remap", "nzcb_prove_logged", "nzcb_memcpy_d2d_async",
    "nzcb_debug_guard_check", "nzcb_debug_guard_selftest", "nzcb_debug_inject_fault", "nzcb_debug_f29",
    "nzcb_msm_table_create_lagrange",
]

NZCB_FAULT_QUOTIENT = 1  # include/nzcb_internal.h
NZCB_DEBUG_GENERIC_K = 2  # include/nzcb_internal.h
NZCB_FAULT_LANE_ALLOC = 3  # include/nzcb_internal.h


def lagrange_commit_enabled() -> bool:
    """Whether prover contexts commit A, B, C over the Lagrange basis (csrc/prover.hip
    lagrange_commit_enabled: NZCB_LAGRANGE_COMMIT unset or non-zero), which decides whether
    the MSM split has Lagrange-basis ranges (nzcb.msmsplit)."""
    import re
    e = os.environ.get("NZCB_LAGRANGE_COMMIT")
    if e is None:
        return True
    m = re.match(r"\s*[+-]?\d+", e)   # as C's atoi: the leading integer, 0 without one
    return bool(m) and int(m.group()) != 0


def guard_check(device: int = -1) -> int:
    """Every guard word past the prover contexts' device buffers on `device` (-1: all) is
    intact; returns how many guards were checked, raises NzcbError listing the damaged
    buffers otherwise (include/nzcb_internal.h nzcb_debug_guard_check)."""
    err, checked, bad = _Err(), c_size_t(0), c_int(0)
    _check(load().nzcb_debug_guard_check(device, ctypes.byref(checked), ctypes.byref(bad), ctypes.byref(err)), err)
    return checked.value


F29_WORDS = {1: (27, 9), 2: (54, 18), 3: (18, 9), 4: (36, 18), 5: (18, 18), 6: (36, 9)}


def f29_check(op: int, words, device: int = 0):
    """Run csrc/f29.h's device product `op` (include/nzcb_internal.h nzcb_debug_f29) over
    items of F29_WORDS[op][0] limb words each; returns the flat list of output words."""
    win, wout = F29_WORDS[op]
    count = len(words) // win
    assert count * win == len(words)
    arr = (c_uint32 * max(1, len(words)))(*words)
    out = (c_uint32 * max(1, count * wout))()
    err = _Err()
    _check(load().nzcb_debug_f29(device, op, arr, count, out, ctypes.byref(err)), err)
    return list(out)[:count * wout]


def guard_selftest(device: int = 0) -> None:
    """A one-word overrun past a fresh guarded buffer is found, and only it."""
    err = _Err()
    _check(load().nzcb_debug_guard_selftest(device, ctypes.byref(err)), err)


class NzcbError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code
        self.name = ERROR_NAMES.get(code, str(code))


class _Err(ctypes.Structure):
    _fields_ = [("code", c_int), ("msg", c_char * 256)]


class NzcpParams(ctypes.Structure):
    """NZCPPubIdentity(IsLive, MaxToBeSignedBytes, MaxCborArrayLenVC, MaxCborMapLenVC, ...)."""
    _fields_ = [("is_live", ctypes.c_int32), ("max_tbs_bytes", ctypes.c_int32),
                ("max_array_len_vc", ctypes.c_int32), ("max_map_len_vc", ctypes.c_int32)]


class NzcpRecord(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("detail", ctypes.c_int32), ("exp", ctypes.c_uint32),
                ("vc_pos", ctypes.c_int32), ("given_len", ctypes.c_int32), ("family_len", ctypes.c_int32),
                ("dob_len", ctypes.c_int32), ("nullifier_len", ctypes.c_int32),
                ("tbs_sha256", c_uint8 * 32), ("nullifier_sha512", c_uint8 * 64), ("nullifier", c_uint8 * 64),
                ("pub", (c_uint8 * 32) * 3)]


# circuits/nzcp_live.circom / nzcp_example.circom mains
NZCP_LIVE = dict(is_live=1, max_tbs_bytes=351, max_array_len_vc=0, max_map_len_vc=4)
NZCP_EXAMPLE = dict(is_live=0, max_tbs_bytes=314, max_array_len_vc=0, max_map_len_vc=4)

LOG_FN = ctypes.CFUNCTYPE(None, c_void_p, ctypes.c_char_p)
# nzcb_ctx_set_msm_split callbacks (include/nzcb.h)
MSM_SEND_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_int, c_void_p, c_size_t)
MSM_GATHER_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_int, POINTER(c_uint8), POINTER(c_uint8))
MSM_LAGRANGE = 0x100   # include/nzcb.h NZCB_MSM_LAGRANGE: the slot's commitment is over the Lagrange basis

_lib = None


def load(path: str | None = None):
    """Load the shared library (raises OSError if it is missing)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # proof lanes and commitment streams need more than HIP's default 4 hardware queues
    # per process (kernels of independent streams sharing a queue serialise); only
    # effective when the HIP runtime has not been initialised yet in this process
    if os.environ.get("GPU_MAX_HW_QUEUES", "4") == "4":  # unset or HIP's default
        os.environ["GPU_MAX_HW_QUEUES"] = "24"
    lib = ctypes.CDLL(path or LIB_PATH)
    u8p = POINTER(c_uint8)
    sigs = {
        "nzcb_version": (ctypes.c_char_p, []),
        "nzcb_device_count": (c_int, []),
        "nzcb_ctx_create": (c_void_p, [u8p, c_size_t, c_int, POINTER(_Err)]),
        "nzcb_ctx_destroy": (None, [c_void_p]),
        "nzcb_ctx_set_logger": (None, [c_void_p, LOG_FN, c_void_p]),
        "nzcb_ctx_set_transcript_public": (None, [c_void_p, c_int]),
        "nzcb_ctx_info": (c_int, [c_void_p, POINTER(c_uint32)]),
        "nzcb_prove": (c_int, [c_void_p, u8p, c_size_t, u8p, u8p, u8p, c_size_t, POINTER(_Err)]),
        "nzcb_prove_witness": (c_int, [c_void_p, u8p, c_size_t, u8p, u8p, u8p, c_size_t, POINTER(_Err)]),
        "nzcb_prove_device": (c_int, [c_void_p, c_void_p, c_size_t, u8p, u8p, u8p, c_size_t, POINTER(_Err)]),
        "nzcb_prove_logged": (c_int, [c_void_p, c_void_p, c_size_t, c_int, u8p, u8p, u8p, c_size_t, LOG_FN, c_void_p,
                                      POINTER(_Err)]),
        "nzcb_ctx_kernel_stats": (c_int, [c_void_p, c_int, POINTER(c_double)]),
        "nzcb_ctx_set_lanes": (c_int, [c_void_p, c_int, POINTER(_Err)]),
        "nzcb_ctx_set_msm_devices": (c_int, [c_void_p, POINTER(c_int), c_int, POINTER(_Err)]),
        "nzcb_vk_from_zkey": (c_int, [u8p, c_size_t, u8p, POINTER(_Err)]),
        "nzcb_vk_from_zkey_file": (c_int, [ctypes.c_char_p, u8p, POINTER(_Err)]),
        "nzcb_vk_to_json": (c_int, [u8p, ctypes.c_char_p, c_size_t]),
        "nzcb_verify": (c_int, [u8p, u8p, u8p, c_int, c_int, POINTER(c_int), POINTER(_Err)]),
        "nzcb_proof_to_calldata": (c_int, [u8p, u8p, c_int, ctypes.c_char_p, c_size_t]),
        "nzcb_vk_to_solidity": (c_int, [u8p, ctypes.c_char_p, c_int, ctypes.c_char_p, c_size_t]),
        "nzcb_engine_lagrange_basis": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_void_p, POINTER(_Err)]),
        "nzcb_ctx_lanes": (c_int, [c_void_p]),
        "nzcb_prove_batch": (c_int, [c_void_p, POINTER(c_void_p), c_size_t, c_int, c_int, u8p, u8p, u8p, c_size_t,
                                     POINTER(_Err)]),
        "nzcb_prove_batch_status": (c_int, [c_void_p, POINTER(c_void_p), c_size_t, c_int, c_int, u8p, u8p, u8p,
                                            c_size_t, POINTER(c_int), POINTER(_Err)]),
        "nzcb_ctx_last_timings": (c_int, [c_void_p, POINTER(c_double), c_int]),
        "nzcb_proof_to_json": (c_int, [u8p, ctypes.c_char_p, c_size_t]),
        "nzcb_public_to_json": (c_int, [u8p, c_int, ctypes.c_char_p, c_size_t]),
        "nzcb_synth_setup": (c_int, [c_int, c_int, c_int, c_uint64, c_uint32, u8p, c_int,
                                     POINTER(POINTER(c_uint8)), POINTER(c_size_t),
                                     POINTER(POINTER(c_uint8)), POINTER(c_size_t), POINTER(_Err)]),
        "nzcb_synth_setup_ex": (c_int, [c_int, c_int, c_int, c_uint64, c_uint32, c_uint32, u8p, c_int,
                                        POINTER(POINTER(c_uint8)), POINTER(c_size_t),
                                        POINTER(POINTER(c_uint8)), POINTER(c_size_t), POINTER(_Err)]),
        "nzcb_free": (None, [c_void_p]),
        "nzcb_engine_create": (c_void_p, [c_int, c_int, c_size_t, POINTER(_Err)]),
        "nzcb_engine_destroy": (None, [c_void_p]),
        "nzcb_engine_ntt": (c_int, [c_void_p, u8p, u8p, c_int, c_int, POINTER(_Err)]),
        "nzcb_engine_msm": (c_int, [c_void_p, u8p, u8p, c_size_t, c_int, u8p, POINTER(_Err)]),
        "nzcb_dev_alloc": (c_void_p, [c_size_t]),
        "nzcb_dev_free": (None, [c_void_p]),
        "nzcb_memcpy_h2d": (c_int, [c_void_p, c_void_p, c_size_t]),
        "nzcb_memcpy_d2h": (c_int, [c_void_p, c_void_p, c_size_t]),
        "nzcb_memcpy_d2d": (c_int, [c_void_p, c_void_p, c_size_t]),
        "nzcb_memcpy_d2d_async": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
        "nzcb_engine_ntt_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, POINTER(_Err)]),
        "nzcb_engine_msm_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_int, u8p, POINTER(_Err)]),
        "nzcb_engine_time_ntt": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, POINTER(c_double),
                                         POINTER(_Err)]),
        "nzcb_engine_fr_mul": (c_int, [c_void_p, u8p, u8p, u8p, c_size_t, c_int, POINTER(_Err)]),
        "nzcb_engine_random_fr": (c_int, [c_void_p, c_void_p, c_size_t, c_uint64, POINTER(_Err)]),
        "nzcb_engine_fixed_base": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p, POINTER(_Err)]),
        "nzcb_engine_time_msm": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_int, c_int, POINTER(c_double),
                                         POINTER(c_double), POINTER(_Err)]),
        "nzcb_engine_msm_fixed_dev": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p, c_size_t, c_int, u8p,
                                              POINTER(_Err)]),
        "nzcb_engine_msm_table_dev": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p, c_size_t, c_int, c_int, c_int,
                                              u8p, POINTER(_Err)]),
        "nzcb_engine_msm_sets_dev": (c_int, [c_void_p, c_void_p, c_size_t, POINTER(c_void_p), c_int, c_size_t, c_int,
                                             u8p, POINTER(_Err)]),
        "nzcb_plonk_setup": (c_int, [ctypes.c_char_p, c_size_t, ctypes.c_char_p, c_size_t, c_int, POINTER(POINTER(c_uint8)),
                                     POINTER(c_size_t), POINTER(_Err)]),
        "nzcb_nzcp_input_signals": (c_size_t, [POINTER(NzcpParams)]),
        "nzcb_nzcp_witness": (c_int, [c_int, POINTER(NzcpParams), u8p, c_int, POINTER(NzcpRecord), POINTER(_Err)]),
        "nzcb_nzcp_witness_dev": (c_int, [c_int, POINTER(NzcpParams), c_void_p, c_int, c_void_p, c_void_p, c_size_t,
                                          c_void_p, POINTER(_Err)]),
        "nzcb_engine_time_msm2": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_int, c_int, c_int,
                                          POINTER(c_double), POINTER(_Err)]),
        "nzcb_ctx_create_devices": (c_void_p, [u8p, c_size_t, POINTER(c_int), c_int, POINTER(_Err)]),
        "nzcb_ctx_devices": (c_int, [c_void_p]),
        "nzcb_ctx_set_msm_split": (c_int, [c_void_p, c_int, c_size_t, c_size_t, MSM_SEND_FN, MSM_GATHER_FN,
                                           c_void_p, POINTER(_Err)]),
        "nzcb_msm_table_create": (c_void_p, [c_int, c_void_p, c_size_t, POINTER(_Err)]),
        "nzcb_msm_table_create_lagrange": (c_void_p, [c_int, c_void_p, c_size_t, c_int, c_size_t, c_size_t,
                                                      POINTER(_Err)]),
        "nzcb_msm_table_run": (c_int, [c_void_p, c_void_p, c_size_t, c_int, u8p, POINTER(_Err)]),
        "nzcb_msm_table_destroy": (None, [c_void_p]),
        "nzcb_ptau_synth": (c_int, [c_int, u8p, c_int, POINTER(POINTER(c_uint8)), POINTER(c_size_t), POINTER(_Err)]),
        "nzcb_wprog_create": (c_void_p, [ctypes.c_char_p, c_size_t, c_int, POINTER(_Err)]),
        "nzcb_wprog_destroy": (None, [c_void_p]),
        "nzcb_wprog_info": (c_int, [c_void_p, POINTER(c_uint32)]),
        "nzcb_wprog_run_dev": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_size_t, POINTER(ctypes.c_int32),
                                       c_void_p, POINTER(_Err)]),
        "nzcb_wprog_run": (c_int, [c_void_p, ctypes.c_char_p, c_int, u8p, POINTER(ctypes.c_int32), POINTER(_Err)]),
        "nzcb_wprog_remap": (c_int, [ctypes.c_char_p, c_size_t, ctypes.c_char_p, c_size_t, ctypes.c_char_p, c_size_t,
                                     POINTER(POINTER(c_uint8)), POINTER(c_size_t), POINTER(c_uint32), POINTER(_Err)]),
        "nzcb_debug_guard_check": (c_int, [c_int, POINTER(c_size_t), POINTER(c_int), POINTER(_Err)]),
        "nzcb_debug_guard_selftest": (c_int, [c_int, POINTER(_Err)]),
        "nzcb_debug_inject_fault": (c_int, [c_void_p, c_int]),
        "nzcb_debug_f29": (c_int, [c_int, c_int, POINTER(c_uint32), c_size_t, POINTER(c_uint32), POINTER(_Err)]),
    }
    lib.missing_symbols = []
    for name, (res, args) in sigs.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            lib.missing_symbols.append(name)
            continue
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _buf(data: bytes):
    return (c_uint8 * len(data)).from_buffer_copy(data) if data else (c_uint8 * 1)()


def _out(n: int):
    return (c_uint8 * max(n, 1))()


def _check(rc: int, err: _Err):
    if rc != 0:
        raise NzcbError(rc, err.msg.decode(errors="replace"))


def version() -> str:
    return load().nzcb_version().decode()


def device_count() -> int:
    return load().nzcb_device_count()


def nzcp_input_signals(params: dict) -> int:
    """Input signals per pass: toBeSigned[8*MaxToBeSignedBytes], toBeSignedLen, data[160]."""
    return load().nzcb_nzcp_input_signals(ctypes.byref(NzcpParams(**params)))


def _record_dict(r: NzcpRecord) -> dict:
    return {
        "status": r.status, "detail": r.detail, "exp": r.exp, "vc_pos": r.vc_pos, "given_len": r.given_len,
        "family_len": r.family_len, "dob_len": r.dob_len, "nullifier_len": r.nullifier_len,
        "tbs_sha256": bytes(r.tbs_sha256), "nullifier_sha512": bytes(r.nullifier_sha512),
        "nullifier": bytes(r.nullifier), "out": [int.from_bytes(bytes(r.pub[k]), "little") for k in range(3)],
    }


def nzcp_witness(inputs: bytes, count: int, params: dict = NZCP_LIVE, device: int = 0) -> list:
    """NZCPPubIdentity witness on the GPU for `count` passes (include/nzcb.h
    nzcb_nzcp_witness). `inputs`: count x nzcp_input_signals(params) x 32-byte LE field
    elements. Returns one dict per pass (status, detail, exp, vc_pos, lengths,
    tbs_sha256, nullifier_sha512, nullifier, out = the 3 public signals as ints)."""
    lib = load()
    prm = NzcpParams(**params)
    need = lib.nzcb_nzcp_input_signals(ctypes.byref(prm)) * 32 * count
    if len(inputs) != need:
        raise ValueError(f"nzcp inputs are {len(inputs)} bytes, expected {need}")
    recs = (NzcpRecord * max(count, 1))()
    err = _Err()
    _check(lib.nzcb_nzcp_witness(device, ctypes.byref(prm), _buf(inputs), count, recs, ctypes.byref(err)), err)
    return [_record_dict(recs[i]) for i in range(count)]


def nzcp_witness_dev(dev_inputs: int, count: int, params: dict = NZCP_LIVE, device: int = 0,
                     dev_records: int | None = None, dev_witness: int | None = None, witness_stride: int = 0,
                     stream: int | None = None):
    """Device-pointer variant (asynchronous on `stream`); see nzcb_nzcp_witness_dev."""
    lib = load()
    err = _Err()
    _check(lib.nzcb_nzcp_witness_dev(device, ctypes.byref(NzcpParams(**params)), dev_inputs, count, dev_records,
                                     dev_witness, witness_stride, stream, ctypes.byref(err)), err)


def nzcp_records_from_bytes(raw: bytes, count: int) -> list:
    size = ctypes.sizeof(NzcpRecord)
    return [_record_dict(NzcpRecord.from_buffer_copy(raw[i * size:(i + 1) * size])) for i in range(count)]


class Engine:
    """Kernel-level access (NTT, MSM, field mul) for tests and microbenchmarks."""

    def __init__(self, device: int = 0, max_log_ntt: int = 12, max_msm_points: int = 1 << 12):
        self.lib = load()
        err = _Err()
        self.h = self.lib.nzcb_engine_create(device, max_log_ntt, max_msm_points, ctypes.byref(err))
        if not self.h:
            raise NzcbError(err.code, err.msg.decode(errors="replace"))

    def close(self):
        if self.h:
            self.lib.nzcb_engine_destroy(self.h)
            self.h = None

    __del__ = close

    def ntt(self, data_lem: bytes, log_n: int, inverse: bool = False) -> bytes:
        n = 1 << log_n
        assert len(data_lem) == 32 * n
        out = _out(32 * n)
        err = _Err()
        _check(self.lib.nzcb_engine_ntt(self.h, _buf(data_lem), out, log_n, int(inverse), ctypes.byref(err)), err)
        return bytes(out)

    def msm(self, bases_lem: bytes, scalars: bytes, scalars_mont: bool = False) -> bytes:
        n = len(scalars) // 32
        assert len(bases_lem) == 64 * n
        out = _out(64)
        err = _Err()
        _check(self.lib.nzcb_engine_msm(self.h, _buf(bases_lem), _buf(scalars), n, int(scalars_mont), out,
                                        ctypes.byref(err)), err)
        return bytes(out)

    def field_mul(self, a_lem: bytes, b_lem: bytes, field_q: bool = False) -> bytes:
        n = len(a_lem) // 32
        out = _out(32 * n)
        err = _Err()
        _check(self.lib.nzcb_engine_fr_mul(self.h, _buf(a_lem), _buf(b_lem), out, n, int(field_q),
                                           ctypes.byref(err)), err)
        return bytes(out)

    def time_ntt(self, dev_in: int, dev_out: int, log_n: int, inverse: bool, reps: int) -> float:
        ms = c_double()
        err = _Err()
        _check(self.lib.nzcb_engine_time_ntt(self.h, dev_in, dev_out, log_n, int(inverse), reps, ctypes.byref(ms),
                                             ctypes.byref(err)), err)
        return ms.value

    def random_fr(self, dev_out: int, n: int, seed: int):
        err = _Err()
        _check(self.lib.nzcb_engine_random_fr(self.h, dev_out, n, seed, ctypes.byref(err)), err)

    def fixed_base(self, dev_scalars: int, n: int, dev_out: int):
        err = _Err()
        _check(self.lib.nzcb_engine_fixed_base(self.h, dev_scalars, n, dev_out, ctypes.byref(err)), err)

    def lagrange_basis(self, dev_ptau: int, ptau_n: int, log_n: int, dev_out: int):
        """dev_out[k] = [L_k(tau)] (k < 2^log_n), then [tau^n] - [1], [tau^(n+1)] - [tau]."""
        err = _Err()
        _check(self.lib.nzcb_engine_lagrange_basis(self.h, dev_ptau, ptau_n, log_n, dev_out, ctypes.byref(err)), err)

    def time_msm(self, dev_bases: int, dev_scalars: int, n: int, scalars_mont: bool, reps: int):
        ms = c_double()
        acc = c_double()
        err = _Err()
        _check(self.lib.nzcb_engine_time_msm(self.h, dev_bases, dev_scalars, n, int(scalars_mont), reps,
                                             ctypes.byref(ms), ctypes.byref(acc), ctypes.byref(err)), err)
        return ms.value, acc.value

    MSM_PHASES = ("keys", "sort", "offsets", "accumulate", "finalize", "reduce", "sums")

    def time_msm_phases(self, dev_bases: int, dev_scalars: int, n: int, scalars_mont: bool, fixed_base: bool,
                        reps: int) -> dict:
        """Wall ms per MSM and HIP-event ms per phase (generic or fixed-base schedule)."""
        out = (c_double * 13)()
        err = _Err()
        _check(self.lib.nzcb_engine_time_msm2(self.h, dev_bases, dev_scalars, n, int(scalars_mont), int(fixed_base),
                                              reps, out, ctypes.byref(err)), err)
        d = {"wall": out[0], "table_build": out[8], "entries": out[9]}
        d.update({k: out[1 + i] for i, k in enumerate(self.MSM_PHASES)})
        d["host_finish"] = out[10]
        d["host_enqueue"] = out[11]     # host time, overlapping the device phases
        d["host_sort_call"] = out[12]
        return d

    def msm_fixed_dev(self, dev_bases: int, n_table: int, dev_scalars: int, n: int, scalars_mont: bool,
                      window: int = 0, sparse: bool = False) -> bytes:
        """Fixed-base (shifted-table) MSM of the first n of n_table device bases; window 0 = the
        PTau tables' default, sparse = the Lagrange table's schedule (msm.hip dyn_chunk)."""
        out = _out(64)
        err = _Err()
        if window or sparse:
            _check(self.lib.nzcb_engine_msm_table_dev(self.h, dev_bases, n_table, dev_scalars, n, int(scalars_mont),
                                                      int(window), int(sparse), out, ctypes.byref(err)), err)
        else:
            _check(self.lib.nzcb_engine_msm_fixed_dev(self.h, dev_bases, n_table, dev_scalars, n, int(scalars_mont),
                                                      out, ctypes.byref(err)), err)
        return bytes(out)

    def msm_sets_dev(self, dev_bases: int, n_table: int, dev_scalars: list, n: int, scalars_mont: bool) -> list:
        """len(dev_scalars) (1..3) MSMs of n scalars over one Lagrange-window table in one schedule
        (the prover's A, B, C commitments): one 64-byte affine result per set."""
        k = len(dev_scalars)
        out = _out(64 * k)
        err = _Err()
        arr = (c_void_p * k)(*dev_scalars)
        _check(self.lib.nzcb_engine_msm_sets_dev(self.h, dev_bases, n_table, arr, k, n, int(scalars_mont), out,
                                                 ctypes.byref(err)), err)
        return [bytes(out)[64 * i:64 * i + 64] for i in range(k)]

    def msm_dev(self, dev_bases: int, dev_scalars: int, n: int, scalars_mont: bool) -> bytes:
        out = _out(64)
        err = _Err()
        _check(self.lib.nzcb_engine_msm_dev(self.h, dev_bases, dev_scalars, n, int(scalars_mont), out,
                                            ctypes.byref(err)), err)
        return bytes(out)


def dev_alloc(nbytes: int) -> int:
    p = load().nzcb_dev_alloc(nbytes)
    if not p:
        raise NzcbError(10, "hipMalloc failed")
    return p


def dev_free(p: int):
    load().nzcb_dev_free(p)


def h2d(dst: int, data: bytes):
    buf = ctypes.create_string_buffer(data, len(data))
    rc = load().nzcb_memcpy_h2d(dst, buf, len(data))
    if rc:
        raise NzcbError(rc, "h2d failed")


def memcpy_h2d_ptr(dst: int, src_addr: int, nbytes: int):
    """Host memory at a raw address (e.g. inside a library-owned zkey buffer) -> device."""
    rc = load().nzcb_memcpy_h2d(dst, src_addr, nbytes)
    if rc:
        raise NzcbError(rc, "h2d failed")


def d2d(dst: int, src: int, nbytes: int):
    if load().nzcb_memcpy_d2d(dst, src, nbytes) != 0:
        raise NzcbError(10, "hipMemcpy D2D failed")


def d2d_async(dst: int, src: int, nbytes: int, stream: int):
    """Device copy ordered on HIP stream `stream` (no host wait)."""
    if load().nzcb_memcpy_d2d_async(dst, src, nbytes, stream) != 0:
        raise NzcbError(10, "hipMemcpyAsync D2D failed")


def d2h(src: int, nbytes: int) -> bytes:
    buf = ctypes.create_string_buffer(nbytes)
    rc = load().nzcb_memcpy_d2h(buf, src, nbytes)
    if rc:
        raise NzcbError(rc, "d2h failed")
    return buf.raw


def _read(x) -> bytes:
    """snarkjs accepts a file name or {type: "mem", data}; here: path, bytes or {"type": "mem", "data": ...}."""
    if isinstance(x, (bytes, bytearray, memoryview)):
        return bytes(x)
    if isinstance(x, dict) and x.get("type") == "mem":
        return bytes(x["data"])
    with open(x, "rb") as f:
        return f.read()


class ProverContext:
    """A zkey uploaded once to one GPU (``nzcb_ctx_create``); prove many witnesses against it."""

    def __init__(self, zkey, device: int = 0, logger=None, transcript_public: bool = True, _raw=None,
                 devices=None):
        """devices: a device set (nzcb_ctx_create_devices): batches spread over all of them,
        single proofs run on devices[0]."""
        self.lib = load()
        self.devices = list(devices) if devices else [device]
        self.device = self.devices[0]
        err = _Err()
        vk = _out(VK_BYTES)
        if _raw is not None:            # (pointer, length) owned by the caller: no host copy
            zptr, zlen = ctypes.cast(_raw[0], POINTER(c_uint8)), _raw[1]
        else:
            data = _read(zkey)
            zptr, zlen = _buf(data), len(data)
        if len(self.devices) > 1:
            devs = (c_int * len(self.devices))(*self.devices)
            self.h = self.lib.nzcb_ctx_create_devices(zptr, zlen, devs, len(self.devices), ctypes.byref(err))
        else:
            self.h = self.lib.nzcb_ctx_create(zptr, zlen, self.device, ctypes.byref(err))
        if not self.h:
            raise NzcbError(err.code, err.msg.decode(errors="replace"))
        verr = _Err()
        _check(self.lib.nzcb_vk_from_zkey(zptr, zlen, vk, ctypes.byref(verr)), verr)
        self.vk = bytes(vk)  # binary verification key (nzcb.verify / vk_to_json)
        info = (c_uint32 * 5)()
        self.lib.nzcb_ctx_info(self.h, info)
        self.domain_size, self.n_public, self.n_vars, self.n_additions, self.n_constraints = list(info)
        self._logcb = None
        if logger is not None:
            self.set_logger(logger)
        if not transcript_public:
            self.lib.nzcb_ctx_set_transcript_public(self.h, 0)

    def set_logger(self, logger):
        fn = getattr(logger, "debug", logger)
        self._logcb = LOG_FN(lambda _u, m: fn(m.decode()))
        self.lib.nzcb_ctx_set_logger(self.h, self._logcb, None)

    def close(self):
        if getattr(self, "h", None):
            self.lib.nzcb_ctx_destroy(self.h)
            self.h = None

    __del__ = close

    def prove_raw(self, wtns, blinding: bytes | None = None):
        """Returns (proof_bytes, public_bytes) in the C-ABI layout. blinding None draws
        random scalars (snarkjs Fr.random(), zero-knowledge); pass fixed bytes, e.g.
        bytes(352), only for reproducible test proofs."""
        data = _read(wtns)
        proof = _out(PROOF_BYTES)
        pub = _out(32 * self.n_public)
        err = _Err()
        bl = _buf(blinding) if blinding is not None else None
        if blinding is not None and len(blinding) != BLINDING_BYTES:
            raise ValueError("blinding must be 11 x 32 bytes")
        _check(self.lib.nzcb_prove(self.h, _buf(data), len(data), bl, proof, pub, 32 * self.n_public,
                                   ctypes.byref(err)), err)
        return bytes(proof), bytes(pub)[:32 * self.n_public]

    def prove_witness_raw(self, witness_le: bytes, blinding: bytes | None = None):
        n = len(witness_le) // 32
        proof = _out(PROOF_BYTES)
        pub = _out(32 * self.n_public)
        err = _Err()
        bl = _buf(blinding) if blinding is not None else None
        _check(self.lib.nzcb_prove_witness(self.h, _buf(witness_le), n, bl, proof, pub, 32 * self.n_public,
                                           ctypes.byref(err)), err)
        return bytes(proof), bytes(pub)[:32 * self.n_public]

    def prove_device_raw(self, dev_witness: int, n_witness: int, blinding: bytes | None = None):
        """Witness already resident in HBM (device pointer, normal-form LE values)."""
        proof = _out(PROOF_BYTES)
        pub = _out(32 * self.n_public)
        err = _Err()
        bl = _buf(blinding) if blinding is not None else None
        _check(self.lib.nzcb_prove_device(self.h, dev_witness, n_witness, bl, proof, pub, 32 * self.n_public,
                                          ctypes.byref(err)), err)
        return bytes(proof), bytes(pub)[:32 * self.n_public]

    def set_lanes(self, lanes: int):
        """Proofs kept in flight by prove_batch (extra lanes share the resident proving key)."""
        err = _Err()
        _check(self.lib.nzcb_ctx_set_lanes(self.h, lanes, ctypes.byref(err)), err)

    def set_msm_devices(self, devices):
        """Split each commitment MSM over these devices (first = the context's device)."""
        arr = (c_int * len(devices))(*devices)
        err = _Err()
        _check(self.lib.nzcb_ctx_set_msm_devices(self.h, arr, len(devices), ctypes.byref(err)), err)

    def set_msm_split(self, world: int, own_points: int, send, gather, own_lagrange: int = 0):
        """Split every commitment MSM across ranks (nzcb_ctx_set_msm_split; nzcb.msmsplit
        builds the callbacks): rank 0 keeps PTau points [0, own_points) and, when
        own_lagrange > 0, Lagrange-basis points [0, own_lagrange) of A, B and C (their slot
        carries MSM_LAGRANGE). send(slot, dev_ptr, count) -> None; gather(slot, own64) ->
        world x 64 bytes. world = 1 restores the local schedule."""
        if world <= 1:
            self._split_cbs = None
            _check(self.lib.nzcb_ctx_set_msm_split(self.h, 1, 0, 0, MSM_SEND_FN(), MSM_GATHER_FN(), None,
                                                   ctypes.byref(_Err())), _Err())
            return

        def _send(_u, slot, ptr, count):
            try:
                send(slot, ptr, count)
                return 0
            except Exception:  # reported through the proof's error
                import traceback
                traceback.print_exc()
                return 1

        def _gather(_u, slot, own, out):
            try:
                parts = gather(slot, ctypes.string_at(own, 64))
                if len(parts) != 64 * world:
                    return 1
                ctypes.memmove(out, parts, len(parts))
                return 0
            except Exception:
                import traceback
                traceback.print_exc()
                return 1

        self._split_cbs = (MSM_SEND_FN(_send), MSM_GATHER_FN(_gather))  # keep alive
        err = _Err()
        _check(self.lib.nzcb_ctx_set_msm_split(self.h, world, own_points, own_lagrange, self._split_cbs[0],
                                               self._split_cbs[1], None, ctypes.byref(err)), err)

    @property
    def lanes(self) -> int:
        return self.lib.nzcb_ctx_lanes(self.h)

    def prove_batch_raw(self, witnesses, n_witness: int | None = None, blindings=None, on_device: bool = False,
                        statuses: list | None = None):
        """Independent proofs over the lanes. witnesses: list of bytes (host) or device
        pointers (on_device). blindings: list of 352-byte values / None. Returns [(proof, pub)].
        With a `statuses` list, a failed proof does not stop the batch: the list receives
        each item's error code (0 = proved; a failed item's bytes are zero) and nothing is
        raised (nzcb_prove_batch_status)."""
        count = len(witnesses)
        keep = []
        ptrs = (c_void_p * max(count, 1))()
        for i, w in enumerate(witnesses):
            if on_device:
                ptrs[i] = w
            else:
                b = _buf(w)
                keep.append(b)
                ptrs[i] = ctypes.cast(b, c_void_p).value
                if n_witness is None:
                    n_witness = len(w) // 32
        bl = None
        if blindings is not None:
            # an item without blinding gets fresh random scalars (snarkjs Fr.random()), never zeros
            bl = _buf(b"".join(x if x is not None else random_blinding() for x in blindings))
        proofs = _out(PROOF_BYTES * count)
        stride = 32 * max(self.n_public, 1)
        pubs = _out(stride * count)
        err = _Err()
        if statuses is None:
            _check(self.lib.nzcb_prove_batch(self.h, ptrs, n_witness or 0, count, int(on_device), bl, proofs, pubs,
                                             stride, ctypes.byref(err)), err)
        else:
            st = (c_int * max(count, 1))()
            rc = self.lib.nzcb_prove_batch_status(self.h, ptrs, n_witness or 0, count, int(on_device), bl, proofs,
                                                  pubs, stride, st, ctypes.byref(err))
            if rc and not any(st[i] for i in range(count)):  # argument errors, before any proof
                _check(rc, err)
            statuses[:] = [st[i] for i in range(count)]
        P, Q = bytes(proofs), bytes(pubs)
        return [(P[i * PROOF_BYTES:(i + 1) * PROOF_BYTES], Q[i * stride:i * stride + 32 * self.n_public])
                for i in range(count)]

    def inject_fault(self, kind: int = NZCB_FAULT_QUOTIENT) -> None:
        """The next proof on each lane perturbs its quotient t (NZCB_FAULT_QUOTIENT: tests of
        the xi check) or takes the grand product's generic k1, k2 path (NZCB_DEBUG_GENERIC_K:
        the same proof), or the next set_lanes growth fails after one new lane
        (NZCB_FAULT_LANE_ALLOC: tests of the rollback); 0 clears it."""
        if self.lib.nzcb_debug_inject_fault(self.h, kind) != 0:
            raise ValueError(f"bad fault kind {kind}")

    def kernel_stats(self, enable: int = -1):
        """MSM bucket-accumulation kernel timing: (ms, launches, points, entries); enable 1/0 resets."""
        out = (c_double * 4)()
        self.lib.nzcb_ctx_kernel_stats(self.h, enable, out)
        return tuple(out)

    def prove(self, wtns, blinding: bytes | None = None):
        """snarkjs-shaped result: {"proof": {...}, "publicSignals": [...]}."""
        proof, pub = self.prove_raw(wtns, blinding)
        return {"proof": proof_to_json(proof), "publicSignals": public_to_json(pub, self.n_public)}

    def last_timings(self):
        """The last proof's phases in ms (include/nzcb.h nzcb_ctx_last_timings): host wall
        clock per round, host time in the MSM calls and enqueueing transforms, and (with
        kernel_stats on) the GPU time of the MSMs and of the transforms."""
        ms = (c_double * 11)()
        k = self.lib.nzcb_ctx_last_timings(self.h, ms, 11)
        names = ["total", "witness", "round1", "round2", "round3", "round4", "round5", "msm_host_wait",
                 "ntt_host_enqueue", "msm_gpu", "ntt_gpu"]
        out = dict(zip(names[:k], list(ms)[:k]))
        return {key: v for key, v in out.items() if v >= 0}


class MsmTable:
    """Resident fixed-base MSM table over device bases (include/nzcb.h nzcb_msm_table_*)."""

    def __init__(self, dev_bases: int, n: int, device: int = 0, _handle=None):
        self.lib = load()
        err = _Err()
        self.n = n
        self.h = _handle or self.lib.nzcb_msm_table_create(device, dev_bases, n, ctypes.byref(err))
        if not self.h:
            raise NzcbError(err.code, err.msg.decode(errors="replace"))

    @classmethod
    def lagrange(cls, dev_ptau: int, ptau_n: int, log_n: int, lo: int, hi: int, device: int = 0):
        """Points [lo, hi) of the Lagrange basis of a 2^log_n domain, from PTau in HBM
        (nzcb_msm_table_create_lagrange): the serving side of the A, B, C commitments."""
        lib = load()
        err = _Err()
        h = lib.nzcb_msm_table_create_lagrange(device, dev_ptau, ptau_n, log_n, lo, hi, ctypes.byref(err))
        if not h:
            raise NzcbError(err.code, err.msg.decode(errors="replace"))
        return cls(0, hi - lo, device, _handle=h)

    def run(self, dev_scalars: int, count: int, scalars_mont: bool = True) -> bytes:
        out = _out(64)
        err = _Err()
        _check(self.lib.nzcb_msm_table_run(self.h, dev_scalars, count, int(scalars_mont), out, ctypes.byref(err)), err)
        return bytes(out)

    def close(self):
        if getattr(self, "h", None):
            self.lib.nzcb_msm_table_destroy(self.h)
            self.h = None

    __del__ = close


class WitnessProgram:
    """A circuit's witness calculator on the GPU (include/nzcb.h nzcb_wprog_*): the
    program written by nzcb.circuit.Circuit.write_program (nzcp_live: nzcb.nzcpgen),
    uploaded once, run for a batch of input vectors, one workgroup per witness."""

    def __init__(self, program: bytes, device: int = 0):
        self.lib = load()
        self.device = device
        err = _Err()
        self.h = self.lib.nzcb_wprog_create(program, len(program), device, ctypes.byref(err))
        if not self.h:
            raise NzcbError(err.code, err.msg.decode(errors="replace"))
        info = (c_uint32 * 5)()
        self.lib.nzcb_wprog_info(self.h, info)
        self.n_wires, self.n_out, self.n_pub_in, self.n_prv_in, self.n_levels = list(info)
        self.n_inputs = self.n_pub_in + self.n_prv_in

    def close(self):
        if getattr(self, "h", None):
            self.lib.nzcb_wprog_destroy(self.h)
            self.h = None

    __del__ = close

    def run(self, inputs: bytes, count: int):
        """Host path: returns (witnesses bytes count x n_wires x 32, statuses)."""
        out = _out(max(1, count * self.n_wires * 32))
        st = (ctypes.c_int32 * max(count, 1))()
        err = _Err()
        _check(self.lib.nzcb_wprog_run(self.h, inputs, count, out, st, ctypes.byref(err)), err)
        return bytes(out)[:count * self.n_wires * 32], [st[i] for i in range(count)]

    def run_dev(self, dev_inputs: int, count: int, dev_witness: int, stride: int) -> list:
        """Device path: witnesses written at dev_witness + i * stride; returns statuses."""
        st = (ctypes.c_int32 * max(count, 1))()
        err = _Err()
        _check(self.lib.nzcb_wprog_run_dev(self.h, dev_inputs, count, dev_witness, stride, st, None,
                                           ctypes.byref(err)), err)
        return [st[i] for i in range(count)]


def wprog_remap(program: bytes, own_sym: bytes, target_sym: bytes) -> bytes:
    """nzcb_wprog_remap: the witness program re-indexed to the wire order of target_sym
    (a circom .sym), matching signals by name against the program's own .sym
    (Circuit.write_sym). Raises NzcbError (unmatched count in .unmatched) when a target
    signal has no counterpart."""
    lib = load()
    out = POINTER(c_uint8)()
    n = c_size_t(0)
    miss = c_uint32(0)
    err = _Err()
    rc = lib.nzcb_wprog_remap(program, len(program), own_sym, len(own_sym), target_sym, len(target_sym),
                              ctypes.byref(out), ctypes.byref(n), ctypes.byref(miss), ctypes.byref(err))
    if rc:
        e = NzcbError(err.code, err.msg.decode(errors="replace"))
        e.unmatched = miss.value
        raise e
    try:
        return ctypes.string_at(out, n.value)
    finally:
        lib.nzcb_free(out)


class NzcpProver:
    """fullProve for nzcp passes on one GPU: the nzcp witness kernel computes each pass's
    public signals (NZCPPubIdentity out[0..2], include/nzcb.h nzcb_nzcp_witness_dev)
    straight into that proof's HBM witness, then nzcb_prove_batch proves them.

    The circuit is a zkey whose public signals are witness[1..3] (snarkjs convention:
    main's outputs first). The rest of each witness is `base_witness` (the nzcp_live
    stand-in of SURVEY.md §8d: a synthetic circuit built with free_public=True, since
    the real r1cs/wasm cannot be built offline). A pass whose witness calculation
    fails raises like circom_runtime's calculateWitness does."""

    def __init__(self, ctx: ProverContext, base_witness: bytes, params: dict = NZCP_LIVE):
        if ctx.n_public != 3:
            raise ValueError("nzcp circuits have 3 public signals")
        self.ctx, self.params = ctx, dict(params)
        self.device = ctx.device
        self.n_witness = len(base_witness) // 32
        self.n_inputs = nzcp_input_signals(self.params)
        self._base = dev_alloc(len(base_witness))
        h2d(self._base, base_witness)
        self._block, self._block_count = None, 0   # per-proof device witnesses, grown on demand
        self._rec = None                          # device records of the same passes
        self._inputs, self._inputs_cap = None, 0

    def close(self):
        for p in (self._block, self._rec, self._base, self._inputs):
            if p:
                dev_free(p)
        self._block = self._rec = self._base = self._inputs = None

    def witness_buffers(self, count: int):
        """Device pointers of `count` witnesses, one contiguous block (stride n_witness x 32 B),
        each initialised from the base witness."""
        stride = self.n_witness * 32
        if count > self._block_count:
            if self._block:
                dev_free(self._block)
                dev_free(self._rec)
            self._block = dev_alloc(stride * count)
            self._rec = dev_alloc(ctypes.sizeof(NzcpRecord) * count)
            for i in range(count):
                d2d(self._block + i * stride, self._base, stride)
            self._block_count = count
        return [self._block + i * stride for i in range(count)]

    def upload_inputs(self, inputs: bytes) -> int:
        """Stage count x n_inputs x 32 B of input signals in HBM; returns the pass count."""
        per = self.n_inputs * 32
        if len(inputs) % per:
            raise ValueError("inputs are not a whole number of passes")
        if len(inputs) > self._inputs_cap:
            if self._inputs:
                dev_free(self._inputs)
            self._inputs, self._inputs_cap = dev_alloc(len(inputs)), len(inputs)
        h2d(self._inputs, inputs)
        return len(inputs) // per

    def witness_staged(self, count: int) -> list:
        """nzcp witness of the staged passes: public signals into witness[1..3] of each
        proof's HBM witness; returns the records. Raises on a failed pass."""
        if count == 0:
            return []
        bufs = self.witness_buffers(count)
        rec_size = ctypes.sizeof(NzcpRecord)
        nzcp_witness_dev(self._inputs, count, self.params, self.device, self._rec, bufs[0], self.n_witness * 32)
        recs = nzcp_records_from_bytes(d2h(self._rec, rec_size * count), count)
        for i, r in enumerate(recs):
            if r["status"] != 0:
                raise NzcbError(r["status"], f"nzcp witness of pass {i} failed: "
                                             f"{NZCP_STATUS.get(r['status'], r['status'])} (detail {r['detail']})")
        return recs

    def full_prove_staged(self, count: int, blindings=None):
        """Witness + proof for the `count` passes staged by upload_inputs (all in HBM).
        Returns ([(proof, public)], records)."""
        recs = self.witness_staged(count)
        res = self.ctx.prove_batch_raw(self.witness_buffers(count), n_witness=self.n_witness, blindings=blindings,
                                       on_device=True)
        return res, recs

    def full_prove(self, inputs: bytes, blindings=None):
        return self.full_prove_staged(self.upload_inputs(inputs), blindings)


NZCP_STATUS = {0: "ok", 1: "toBeSigned bit check", 2: "toBeSignedLen > MaxToBeSignedBytes",
               3: "LessThan operands out of range", 4: "QuinSelector index out of range",
               5: "CBOR type is not a map", 6: "CBOR map length > 23", 7: "CBOR type is not a string",
               8: "negative toBeSignedLen (unpinned)"}


def proof_to_json(proof: bytes) -> dict:
    lib = load()
    cap = 8192
    out = ctypes.create_string_buffer(cap)
    rc = lib.nzcb_proof_to_json(_buf(proof), out, cap)
    if rc:
        raise NzcbError(1, "json buffer too small")
    return json.loads(out.value.decode())


def public_to_json(pub: bytes, n_public: int) -> list:
    lib = load()
    cap = 80 * n_public + 8
    out = ctypes.create_string_buffer(cap)
    rc = lib.nzcb_public_to_json(_buf(pub), n_public, out, cap)
    if rc:
        raise NzcbError(1, "json buffer too small")
    return json.loads(out.value.decode())


def _json_text(fn, *args) -> str:
    need = fn(*args, None, 0)
    out = ctypes.create_string_buffer(max(need, 1))
    rc = fn(*args, out, max(need, 1))
    if rc != 0:
        raise NzcbError(11, "json encoding failed")
    return out.value.decode()


def vk_from_zkey(zkey) -> bytes:
    """Binary verification key (include/nzcb.h NZCB_VK_BYTES) of a zkey: bytes, a path, or
    a (pointer, length) library buffer (nzcb.plonk_setup_raw)."""
    out = _out(VK_BYTES)
    err = _Err()
    if isinstance(zkey, str):   # memory-mapped by the library (zkeys past 2 GiB)
        _check(load().nzcb_vk_from_zkey_file(zkey.encode(), out, ctypes.byref(err)), err)
        return bytes(out)
    if isinstance(zkey, tuple):
        ptr, size = ctypes.cast(zkey[0], POINTER(c_uint8)), zkey[1]
    else:
        ptr, size = _buf(zkey), len(zkey)
    _check(load().nzcb_vk_from_zkey(ptr, size, out, ctypes.byref(err)), err)
    return bytes(out)


def vk_to_json(vk: bytes) -> dict:
    """snarkjs verification_key.json object."""
    import json
    return json.loads(_json_text(load().nzcb_vk_to_json, _buf(vk)))


def _le(x) -> bytes:
    return int(x).to_bytes(32, "little")


def vk_from_json(obj: dict) -> bytes:
    """verification_key.json (snarkjs layout) -> binary verification key."""
    def g1(p):
        return bytes(64) if str(p[2]) == "0" else _le(p[0]) + _le(p[1])

    out = int(obj["nPublic"]).to_bytes(4, "little") + int(obj["power"]).to_bytes(4, "little")
    out += _le(obj["k1"]) + _le(obj["k2"])
    out += b"".join(g1(obj[k]) for k in VK_POINTS)
    (x0, x1), (y0, y1) = obj["X_2"][0], obj["X_2"][1]
    out += _le(x0) + _le(x1) + _le(y0) + _le(y1) + _le(obj["w"])
    return out


def proof_from_json(obj: dict) -> bytes:
    """snarkjs proof object -> NZCB_PROOF_BYTES."""
    def g1(p):
        return bytes(64) if str(p[2]) == "0" else _le(p[0]) + _le(p[1])

    return b"".join(g1(obj[k]) for k in PROOF_POINTS) + b"".join(_le(obj[k]) for k in PROOF_EVALS)


def verify(vk: bytes, proof: bytes, public: bytes, transcript_public: bool = True) -> bool:
    """Pairing verification of a binary proof; public = nPublic x 32-byte LE."""
    valid = c_int(0)
    err = _Err()
    _check(load().nzcb_verify(_buf(vk), _buf(proof), _buf(public), len(public) // 32, int(transcript_public),
                              ctypes.byref(valid), ctypes.byref(err)), err)
    return bool(valid.value)


def proof_to_calldata(proof: bytes, public: bytes) -> str:
    """snarkjs `zkey export soliditycalldata` text for a PLONK proof."""
    return _json_text(load().nzcb_proof_to_calldata, _buf(proof), _buf(public), len(public) // 32)


def vk_to_solidity(vk: bytes, contract_name: str = "PlonkVerifier", transcript_public: bool = True) -> str:
    """snarkjs `zkey export solidityverifier`: the Solidity PLONK verifier of a binary
    verification key (include/nzcb.h nzcb_vk_to_solidity)."""
    fn = load().nzcb_vk_to_solidity
    name = contract_name.encode()
    need = fn(_buf(vk), name, int(transcript_public), None, 0)
    if need < 0:
        raise NzcbError(1, f"solidity verifier: bad verification key or contract name {contract_name!r}")
    out = ctypes.create_string_buffer(need)
    if fn(_buf(vk), name, int(transcript_public), out, need) != 0:
        raise NzcbError(11, "solidity verifier: rendering failed")
    return out.value.decode()


class plonk:
    """snarkjs-compatible entry points (``snarkjs.plonk.prove`` / ``verify`` [EXT])."""

    @staticmethod
    def verify(vk_verifier: dict, publicSignals, proof: dict, transcript_public: bool = True) -> bool:
        """snarkjs.plonk.verify(vkey, publicSignals, proof) on the JSON objects."""
        pub = b"".join(_le(x) for x in publicSignals)
        return verify(vk_from_json(vk_verifier), proof_from_json(proof), pub, transcript_public)

    @staticmethod
    def prove(zkeyFileName, witnessFileName, logger=None, device: int = 0, blinding: bytes | None = None):
        ctx = ProverContext(zkeyFileName, device=device, logger=logger)
        try:
            if blinding is None:
                blinding = random_blinding()
            return ctx.prove(witnessFileName, blinding)
        finally:
            ctx.close()


def random_blinding() -> bytes:
    """11 uniform Fr scalars (snarkjs ``Fr.random()``), 32-byte LE each."""
    import secrets
    r = 21888242871839275222246405745257275088548364400416034343698204186575808495617
    return b"".join((secrets.randbelow(r)).to_bytes(32, "little") for _ in range(11))


SYNTH_FREE_PUBLIC = 1


def _synth_raw(power, n_public, n_inputs, seed, n_constraints, tau, device, free_public):
    lib = load()
    zp = POINTER(c_uint8)()
    wp = POINTER(c_uint8)()
    zl = c_size_t()
    wl = c_size_t()
    err = _Err()
    taub = _buf(int(tau).to_bytes(32, "little"))
    flags = SYNTH_FREE_PUBLIC if free_public else 0
    _check(lib.nzcb_synth_setup_ex(power, n_public, n_inputs, seed, n_constraints, flags, taub, device,
                                   ctypes.byref(zp), ctypes.byref(zl), ctypes.byref(wp), ctypes.byref(wl),
                                   ctypes.byref(err)), err)
    return zp, zl.value, wp, wl.value


def synth_context(power: int, n_public: int = 3, n_inputs: int = 8, seed: int = 0x6E7A6362,
                  n_constraints: int = 0, tau: int = 0x6E7A6362746175, device: int = 0, free_public: bool = False):
    """Build the synthetic circuit's zkey on `device` and upload it straight into a
    ProverContext without copying the (multi-GB) zkey through Python. Returns (ctx, wtns bytes).
    free_public: public signals on their public-input gate only (NZCB_SYNTH_FREE_PUBLIC)."""
    lib = load()
    zp, zl, wp, wl = _synth_raw(power, n_public, n_inputs, seed, n_constraints, tau, device, free_public)
    try:
        ctx = ProverContext(None, device=device, _raw=(zp, zl))
        wtns = _take(wp, wl)
    finally:
        lib.nzcb_free(ctypes.cast(zp, c_void_p))
        lib.nzcb_free(ctypes.cast(wp, c_void_p))
    return ctx, wtns


def synth_setup(power: int, n_public: int = 3, n_inputs: int = 8, seed: int = 0x6E7A6362,
                n_constraints: int = 0, tau: int = 0x6E7A6362746175, device: int = 0, free_public: bool = False):
    """Seeded synthetic circuit + zkey built on the GPU (``nzcb_synth_setup_ex``). Returns (zkey, wtns) bytes."""
    lib = load()
    zp, zl, wp, wl = _synth_raw(power, n_public, n_inputs, seed, n_constraints, tau, device, free_public)
    try:
        zkey = _take(zp, zl)
        wtns = _take(wp, wl)
    finally:
        lib.nzcb_free(ctypes.cast(zp, c_void_p))
        lib.nzcb_free(ctypes.cast(wp, c_void_p))
    return zkey, wtns


def plonk_setup(r1cs: bytes, ptau: bytes, device: int = 0) -> bytes:
    """snarkjs ``plonk setup <r1cs> <ptau> <zkey>`` (snarkjs 0.4.12 plonk_setup.js, run at
    /root/reference/Makefile:55,60): returns the PLONK zkey bytes. The NTTs and the
    commitments run on `device`; raises NzcbError as snarkjs throws (curve mismatch,
    "circuit too big for this power of tau ceremony", "Variable not used")."""
    ptr, size = plonk_setup_raw(r1cs, ptau, device)
    try:
        return _take(ptr, size)
    finally:
        load().nzcb_free(ptr)


def plonk_setup_raw(r1cs: bytes, ptau: bytes, device: int = 0):
    """plonk_setup returning the library-owned zkey buffer (pointer, length) without a
    host copy (a 2^21 zkey is about 3.9 GB); release with nzcb.free_ptr."""
    lib = load()
    zp = POINTER(c_uint8)()
    zl = c_size_t()
    err = _Err()
    _check(lib.nzcb_plonk_setup(bytes(r1cs), len(r1cs), bytes(ptau), len(ptau), device, ctypes.byref(zp),
                                ctypes.byref(zl), ctypes.byref(err)), err)
    return ctypes.cast(zp, c_void_p).value, zl.value


def free_ptr(ptr: int):
    load().nzcb_free(ptr)


def _take(ptr, size: int) -> bytes:
    """bytes of a library buffer (ctypes.string_at takes an int size, < 2 GiB)."""
    addr = ctypes.cast(ptr, c_void_p).value if not isinstance(ptr, int) else ptr
    return bytes((c_uint8 * size).from_address(addr)) if size else b""


def ptau_synth(power: int, tau: int, device: int = 0) -> bytes:
    """Powers-of-tau file (snarkjs layout, sections 1-3) for a trapdoor tau, built on the
    GPU (include/nzcb.h nzcb_ptau_synth)."""
    lib = load()
    pp = POINTER(c_uint8)()
    pl = c_size_t()
    err = _Err()
    _check(lib.nzcb_ptau_synth(power, _buf(int(tau).to_bytes(32, "little")), device, ctypes.byref(pp),
                               ctypes.byref(pl), ctypes.byref(err)), err)
    try:
        return _take(pp, pl.value)
    finally:
        lib.nzcb_free(pp)


def synth_setup_raw(power: int, n_public: int = 3, n_inputs: int = 8, seed: int = 0x6E7A6362,
                    n_constraints: int = 0, tau: int = 0x6E7A6362746175, device: int = 0, free_public: bool = False):
    """Like synth_setup but returns library-owned host buffers (zkey_ptr, zkey_len, wtns_ptr, wtns_len)
    without copying them into Python; release with free_raw()."""
    zp, zl, wp, wl = _synth_raw(power, n_public, n_inputs, seed, n_constraints, tau, device, free_public)
    return (ctypes.cast(zp, c_void_p).value, zl, ctypes.cast(wp, c_void_p).value, wl)


def free_raw(raw):
    lib = load()
    lib.nzcb_free(raw[0])
    lib.nzcb_free(raw[2])
