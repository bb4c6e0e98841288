"""nzcp_live end to end: the circuit's r1cs and witness program (nzcb.nzcpgen), its PLONK
zkey (``snarkjs plonk setup nzcp_live.r1cs powersOfTau28_hez_final_21.ptau``,
/root/reference/Makefile:59-62, with a seeded-tau ptau in place of the ceremony file), and
``NzcpLiveProver``: plonk.fullProve for a batch of passes with every witness signal
computed on the GPU (nzcb_wprog_run_dev) and proved by nzcb_prove_batch, all in HBM.

The signal order is this build's (nzcb.nzcpgen docstring), so parity of the proof bytes
against snarkjs on the real zkey is unpinned; the public signals are pinned by the
reference's test vectors through oracle/nzcp_circuit.py.
"""
from __future__ import annotations

import hashlib
import os

from . import circuit, nzcpgen

TAU = 0x6E7A6362746175          # SURVEY.md §8d seeded trapdoor (bench.py TAU)
_HERE = os.path.dirname(os.path.abspath(__file__))


def _source_hash() -> str:
    h = hashlib.sha256()
    for f in ("circuit.py", "nzcpgen.py"):
        with open(os.path.join(_HERE, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _cache_dir() -> str | None:
    d = os.environ.get("NZCB_CACHE_DIR", os.path.join(os.path.expanduser("~"), ".cache", "nzcb"))
    try:
        os.makedirs(d, exist_ok=True)
        return d
    except OSError:
        return None


def build(params: dict = nzcpgen.LIVE, cache: bool = True):
    """(r1cs bytes, witness program bytes, Circuit or None) of NZCPPubIdentity(params);
    cached on disk by generator-source hash (the Circuit object only when generated)."""
    key = f"nzcp_{params['is_live']}_{params['max_tbs_bytes']}_{params['max_array_len_vc']}_" \
          f"{params['max_map_len_vc']}_{_source_hash()}"
    d = _cache_dir() if cache else None
    if d:
        rp, pp = os.path.join(d, key + ".r1cs"), os.path.join(d, key + ".wprog")
        if os.path.exists(rp) and os.path.exists(pp):
            with open(rp, "rb") as f:
                r1cs = f.read()
            with open(pp, "rb") as f:
                prog = f.read()
            return r1cs, prog, None
    c = nzcpgen.nzcp_pub_identity(**params)
    r1cs, prog = c.write_r1cs(), c.write_program()
    if d:
        for path, data in ((rp, r1cs), (pp, prog)):
            tmp = f"{path}.{os.getpid()}.tmp"
            with open(tmp, "wb") as f:
                f.write(data)
            os.replace(tmp, path)
    return r1cs, prog, c


def write_artifacts(out_dir: str, params: dict = nzcpgen.LIVE, name: str = "nzcp_live") -> dict:
    """The compiler outputs circom would write for the circuit, from this build's generator:
    <name>.r1cs (circom --r1cs), <name>.nzwp (the GPU witness program, in place of
    <name>.wasm) and <name>.nzwp.sym (circom --sym layout: "label,wire,component,name"),
    the own .sym that nzcb_wprog_remap / wtns.remapProgram match against circom's
    <name>.sym. Returns {kind: path}."""
    c = nzcpgen.nzcp_pub_identity(**params)
    os.makedirs(out_dir, exist_ok=True)
    out = {}
    for kind, ext, data in (("r1cs", ".r1cs", c.write_r1cs()), ("program", ".nzwp", c.write_program()),
                            ("sym", ".nzwp.sym", c.write_sym())):
        path = os.path.join(out_dir, name + ext)
        with open(path, "wb") as f:
            f.write(data)
        out[kind] = path
    return out


PTAU_POWER = 21                 # powersOfTau28_hez_final_21.ptau (/root/reference/README.md:40)


def setup_raw(r1cs: bytes, tau: int = TAU, device: int = 0, ptau_power: int = PTAU_POWER):
    """PLONK zkey of the r1cs (nzcb_plonk_setup) against a seeded-tau ptau of the
    reference's ceremony power, as a library-owned (pointer, length) buffer (release with
    nzcb.free_ptr); raises like snarkjs if the circuit does not fit."""
    import nzcb
    return nzcb.plonk_setup_raw(r1cs, nzcb.ptau_synth(ptau_power, tau, device), device)


def context(r1cs: bytes, tau: int = TAU, device: int = 0):
    """(ProverContext on the zkey, the zkey's raw buffer) without copying the zkey through
    Python; the caller frees the buffer with nzcb.free_ptr once it no longer needs it."""
    import nzcb
    raw = setup_raw(r1cs, tau, device)
    try:
        ctx = nzcb.ProverContext(None, device=device, _raw=raw)
    except Exception:
        nzcb.free_ptr(raw[0])
        raise
    return ctx, raw


class NzcpLiveProver:
    """plonk.fullProve for nzcp passes on one GPU with the real circuit: the witness
    program computes every signal of each pass's witness in HBM, then nzcb_prove_batch
    proves them over the context's lanes (SURVEY.md §8a rows a1-a2 + a3-a12)."""

    def __init__(self, ctx, program: bytes):
        import nzcb
        self.nzcb = nzcb
        self.ctx = ctx
        self.wp = nzcb.WitnessProgram(program, ctx.device)
        if ctx.n_public != self.wp.n_out + self.wp.n_pub_in:
            raise ValueError("witness program and zkey disagree on the public signals")
        if ctx.n_vars - ctx.n_additions != self.wp.n_wires:
            raise ValueError(f"witness program has {self.wp.n_wires} wires, zkey expects "
                             f"{ctx.n_vars - ctx.n_additions}")
        self.n_witness = self.wp.n_wires
        self._block, self._block_count = None, 0
        self._inputs, self._inputs_cap = None, 0

    def close(self):
        for p in (self._block, self._inputs):
            if p:
                self.nzcb.dev_free(p)
        self._block = self._inputs = None
        self.wp.close()

    def witness_buffers(self, count: int) -> list:
        stride = self.n_witness * 32
        if count > self._block_count:
            if self._block:
                self.nzcb.dev_free(self._block)
            self._block = self.nzcb.dev_alloc(stride * count)
            self._block_count = count
        return [self._block + i * stride for i in range(count)]

    def upload_inputs(self, inputs: bytes) -> int:
        per = self.wp.n_inputs * 32
        if len(inputs) % per:
            raise ValueError("inputs are not a whole number of passes")
        if len(inputs) > self._inputs_cap:
            if self._inputs:
                self.nzcb.dev_free(self._inputs)
            self._inputs, self._inputs_cap = self.nzcb.dev_alloc(len(inputs)), len(inputs)
        self.nzcb.h2d(self._inputs, inputs)
        return len(inputs) // per

    def witness_staged(self, count: int) -> list:
        """Full witnesses of the staged passes in HBM; raises on a failed pass (like
        circom_runtime's calculateWitness)."""
        if count == 0:
            return []
        bufs = self.witness_buffers(count)
        st = self.wp.run_dev(self._inputs, count, bufs[0], self.n_witness * 32)
        for i, s in enumerate(st):
            if s:
                raise self.nzcb.NzcbError(s, f"nzcp witness of pass {i} failed: "
                                             f"{self.nzcb.NZCP_STATUS.get(s, s)}")
        return bufs

    def full_prove_staged(self, count: int, blindings=None):
        bufs = self.witness_staged(count)
        return self.ctx.prove_batch_raw(bufs, n_witness=self.n_witness, blindings=blindings, on_device=True)

    def full_prove(self, inputs: bytes, blindings=None):
        return self.full_prove_staged(self.upload_inputs(inputs), blindings)

    def witness_bytes(self, index: int) -> bytes:
        """One staged witness copied back (tests)."""
        return self.nzcb.d2h(self._block + index * self.n_witness * 32, self.n_witness * 32)


def wtns_file(witness_le: bytes) -> bytes:
    """snarkjs .wtns (version 2) of a normal-form LE witness."""
    import struct
    n = len(witness_le) // 32
    hdr = struct.pack("<I", 32) + circuit.R.to_bytes(32, "little") + struct.pack("<I", n)
    return circuit._binfile(b"wtns", 2, [(1, hdr), (2, witness_le)])
