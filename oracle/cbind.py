"""ctypes binding of oracle/c/nzcb_ref.c (multi-threaded CPU restatement of the prover).

TEST INFRASTRUCTURE ONLY (see oracle/bn254.py header): the checker for large
sizes and bench.py's ``cpu_baseline`` (kind "port"). Parity unpinned vs snarkjs.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import time

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libnzcb_ref.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "c")], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        lib.nzcb_ref_prove.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, u8p, ctypes.c_int, ctypes.c_int,
                                       u8p, u8p, ctypes.POINTER(ctypes.c_double), ctypes.c_char_p]
        lib.nzcb_ref_msm.argtypes = [u8p, u8p, ctypes.c_size_t, ctypes.c_int, u8p]
        lib.nzcb_ref_ntt.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        _lib = lib
    return _lib


def _buf(b: bytes):
    return (ctypes.c_uint8 * max(len(b), 1)).from_buffer_copy(b if b else b"\0")


def default_threads() -> int:
    """Every core this process may use: the CPU affinity set, capped by OMP_NUM_THREADS
    when the host exports it (the GPU box shows the whole machine in nproc / affinity but
    leases 16 cores per GPU and exports OMP_NUM_THREADS=16 to say so)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def threads_reason(th: int) -> str:
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) == th:
        return f"{th} threads = the lease's CPU share (OMP_NUM_THREADS={omp})"
    return f"{th} threads = every core in the process's CPU affinity set"


def prove(zkey, wtns, blinding: bytes | None = None, transcript_pub: bool = True,
          threads: int | None = None, npub: int = 64):
    """zkey / wtns: bytes, or (pointer, length) pairs of host memory owned by the caller.
    Returns (proof_bytes, public_bytes, times{total,msm,ntt} seconds)."""
    lib = load()
    proof = (ctypes.c_uint8 * 800)()
    pub = (ctypes.c_uint8 * (32 * npub))()
    times = (ctypes.c_double * 3)()
    err = ctypes.create_string_buffer(256)
    bl = _buf(blinding) if blinding is not None else None
    u8p = ctypes.POINTER(ctypes.c_uint8)

    def arg(x):
        if isinstance(x, tuple):
            return ctypes.cast(x[0], u8p), x[1]
        return _buf(x), len(x)

    zp, zl = arg(zkey)
    wp, wl = arg(wtns)
    rc = lib.nzcb_ref_prove(zp, zl, wp, wl, bl, int(transcript_pub), threads or default_threads(), proof, pub,
                            times, err)
    if rc:
        raise RuntimeError(err.value.decode())
    return bytes(proof), bytes(pub), {"total": times[0], "msm": times[1], "ntt": times[2]}


def msm(bases_lem: bytes, scalars_lem: bytes, threads: int | None = None) -> bytes:
    lib = load()
    out = (ctypes.c_uint8 * 64)()
    lib.nzcb_ref_msm(_buf(bases_lem), _buf(scalars_lem), len(scalars_lem) // 32, threads or default_threads(), out)
    return bytes(out)


def timed_sample(power: int, threads: int | None = None):
    """bench.py cpu_baseline: one full proof of the same synthetic nzcp_live workload on
    `threads` host cores (zkey built by the GPU library's setup, proved by the C port)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "nzcb-circom_amd"))
    import nzcb
    th = threads or default_threads()
    raw = nzcb.synth_setup_raw(power, 3, 2970, 0x6E7A6362, 0, 0x6E7A6362746175)
    try:
        t0 = time.time()
        _, _, t = prove((raw[0], raw[1]), (raw[2], raw[3]), bytes(352), True, th, 3)
    finally:
        nzcb.free_raw(raw)
    wall = time.time() - t0
    return {"value": round(1.0 / wall, 5), "unit": "proofs/s", "cores": th, "kind": "port",
            "sample": f"1 full proof, n=2^{power} synthetic nzcp_live, oracle/c/nzcb_ref.c on {threads_reason(th)} "
                      f"({wall:.1f} s; msm {t['msm']:.1f} s, ntt {t['ntt']:.1f} s)"}


def timed_prove(zkey, wtns, what: str, threads: int | None = None):
    """bench.py cpu_baseline: one full proof of the given zkey ((pointer, length) or bytes)
    and wtns on `threads` host cores."""
    th = threads or default_threads()
    t0 = time.time()
    _, _, t = prove(zkey, wtns, bytes(352), True, th, 3)
    wall = time.time() - t0
    return {"value": round(1.0 / wall, 5), "unit": "proofs/s", "cores": th, "kind": "port",
            "sample": f"{what}, oracle/c/nzcb_ref.c on {threads_reason(th)} "
                      f"({wall:.1f} s; msm {t['msm']:.1f} s, ntt {t['ntt']:.1f} s)"}
