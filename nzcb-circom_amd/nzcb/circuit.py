"""R1CS circuit builder and witness-program emitter (the compiler half of circom).

The reference compiles its circuit with ``circom --r1cs --wasm --O2``
(/root/reference/Makefile:12-13) and computes witnesses with the circom wasm runtime
(circom_runtime 0.1.17, /root/reference/yarn.lock:2496). Neither is on disk, so
this module plays both roles for the circuits written in ``nzcb.nzcpgen``:

* it allocates signals (wire 0 = the constant 1, then outputs, public inputs, private
  inputs, intermediate signals: circom's wire order) and records constraints
  ``A * B = C`` over linear combinations, written as an iden3 r1cs file that
  ``nzcb_plonk_setup`` (snarkjs ``plonk setup``) turns into a zkey;
* it records, for every intermediate signal, how the witness calculator computes it:
  a **witness program** that the GPU runs (``csrc/wvm.hip``, C-ABI ``nzcb_wprog_*``).

Linear combinations are dicts ``{wire: coef}`` (coefficients mod r, wire 0 for the
constant). Signals are assigned in creation order, which is a topological order;
``write_program`` groups the operations into dependency levels, each of which the GPU
executes in parallel.

Witness operations (``OP_*``), the contract shared with ``csrc/wvm.hip``:

  LIN    dst = A
  MUL    dst = A * B + C
  INV    dst = 1 / A, or 0 when A = 0 (circomlib IsZero's ``inv <-- in != 0 ? 1/in : 0``)
  BITS   dst[0..n) = the n low bits of A (circomlib Num2Bits ``out[i] <-- (in >> i) & 1``);
         fails with ``err`` when A >= 2^n (the constraint ``lc1 === in`` would not hold)
  CHECK  fails with ``err`` unless A = 0, or A * B = 0 when B is given (a ``===``
         constraint or an ``assert``)
  QUIN   QuinSelector(n) core (quinSelector.circom:27-38): index A, inputs in[k] = wire
         b_off + k for k < m = b_n and 0 past m; writes eq[0..n), inv[0..n), sums[0..m)
  SHA256 one SHA-256 compression (layout: ``sha_block_layout``)
  SHA512 SHA-512 of exactly 64 message bytes (one block, constant padding)

A failing op records (its creation order, err); the lowest creation order wins, so the
reported failure is the first in template order, as circom's witness calculator
throws at the first failed check.
"""
from __future__ import annotations

import contextlib
import struct

R = 21888242871839275222246405745257275088548364400416034343698204186575808495617

OP_LIN, OP_MUL, OP_INV, OP_BITS, OP_CHECK, OP_QUIN, OP_SHA256, OP_SHA512 = range(8)
MACRO_OPS = (OP_QUIN, OP_SHA256, OP_SHA512)
NO_WIRE = 0xFFFFFFFF
PROGRAM_MAGIC = b"nzwp"
PROGRAM_VERSION = 2


def lc(x) -> dict:
    """Coerce an int (constant) or dict into a fresh linear combination."""
    if isinstance(x, dict):
        return dict(x)
    x %= R
    return {0: x} if x else {}


def w(wire: int) -> dict:
    return {wire: 1}


def add(*xs) -> dict:
    out = {}
    for x in xs:
        if isinstance(x, int):
            if x % R:
                out[0] = (out.get(0, 0) + x) % R
            continue
        for k, v in x.items():
            out[k] = (out.get(k, 0) + v) % R
    return {k: v for k, v in out.items() if v}


def scale(x, c: int) -> dict:
    if isinstance(x, int):
        return lc(x * c)
    c %= R
    if c == 0:
        return {}
    return {k: v * c % R for k, v in x.items()}


def sub(a, b) -> dict:
    return add(a, scale(b, -1))


def is_const(x) -> bool:
    return isinstance(x, int) or all(k == 0 for k in x)


def const_value(x) -> int:
    return x % R if isinstance(x, int) else x.get(0, 0)


# ---------------------------------------------------------------------------------
# SHA-2 block layouts, shared by the gadgets (nzcpgen), the GPU writer (csrc/wvm.hip)
# and the CPU evaluator (oracle/wvm.py)
# ---------------------------------------------------------------------------------
SHA256_SPEC = dict(bits=32, rounds=64, S0=(2, 13, 22), S1=(6, 11, 25), s0=(7, 18, 3), s1=(17, 19, 10))
SHA512_SPEC = dict(bits=64, rounds=80, S0=(28, 34, 39), S1=(14, 18, 41), s0=(1, 8, 7), s1=(19, 61, 6))


def xor_kinds(bits: int, r1: int, r2: int, r3: int, shr_last: bool):
    """Per output bit i of ROTR r1 ^ ROTR r2 ^ (SHR|ROTR) r3: 3 (XOR3: mid, p) or 2 (XOR2: m)."""
    return [2 if shr_last and i + r3 >= bits else 3 for i in range(bits)]


def sha_block_layout(spec: dict) -> dict:
    """Offsets (signals from the block's base wire) of one SHA-2 compression:

      schedule t = 16..R-1: sigma0(W[t-15]) xor signals, sigma1(W[t-2]) xor signals,
                            W[t] = 32|64 bits (LSB first) + 2 carry bits
      round t = 0..R-1:     Sigma1(e) xor signals, ch q[bits], Sigma0(a) xor signals,
                            maj (mid, q)[bits], new a bits + 3 carries, new e bits + 3 carries
      final:                H_out[j] = H_in[j] + V[j]: bits + 1 carry, j = 0..7

    XOR3 bits hold (mid = b c, p = a (1 - 2b - 2c + 4 mid)); XOR2 bits hold m = a b."""
    B = spec["bits"]
    s0 = xor_kinds(B, *spec["s0"], True)
    s1 = xor_kinds(B, *spec["s1"], True)
    S = [3] * B
    nx = lambda kinds: sum(2 if k == 3 else 1 for k in kinds)  # noqa: E731
    sched = nx(s0) + nx(s1) + B + 2
    rnd = nx(S) + B + nx(S) + 2 * B + (B + 3) + (B + 3)
    n_sched = spec["rounds"] - 16
    size = n_sched * sched + spec["rounds"] * rnd + 8 * (B + 1)
    return dict(s0_kinds=s0, s1_kinds=s1, sched=sched, round=rnd, sched_base=0,
                round_base=n_sched * sched, final_base=n_sched * sched + spec["rounds"] * rnd,
                size=size, bits=B)


SHA256_K = [
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2]
SHA256_IV = [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19]
SHA512_K = [
    0x428a2f98d728ae22, 0x7137449123ef65cd, 0xb5c0fbcfec4d3b2f, 0xe9b5dba58189dbbc, 0x3956c25bf348b538,
    0x59f111f1b605d019, 0x923f82a4af194f9b, 0xab1c5ed5da6d8118, 0xd807aa98a3030242, 0x12835b0145706fbe,
    0x243185be4ee4b28c, 0x550c7dc3d5ffb4e2, 0x72be5d74f27b896f, 0x80deb1fe3b1696b1, 0x9bdc06a725c71235,
    0xc19bf174cf692694, 0xe49b69c19ef14ad2, 0xefbe4786384f25e3, 0x0fc19dc68b8cd5b5, 0x240ca1cc77ac9c65,
    0x2de92c6f592b0275, 0x4a7484aa6ea6e483, 0x5cb0a9dcbd41fbd4, 0x76f988da831153b5, 0x983e5152ee66dfab,
    0xa831c66d2db43210, 0xb00327c898fb213f, 0xbf597fc7beef0ee4, 0xc6e00bf33da88fc2, 0xd5a79147930aa725,
    0x06ca6351e003826f, 0x142929670a0e6e70, 0x27b70a8546d22ffc, 0x2e1b21385c26c926, 0x4d2c6dfc5ac42aed,
    0x53380d139d95b3df, 0x650a73548baf63de, 0x766a0abb3c77b2a8, 0x81c2c92e47edaee6, 0x92722c851482353b,
    0xa2bfe8a14cf10364, 0xa81a664bbc423001, 0xc24b8b70d0f89791, 0xc76c51a30654be30, 0xd192e819d6ef5218,
    0xd69906245565a910, 0xf40e35855771202a, 0x106aa07032bbd1b8, 0x19a4c116b8d2d0c8, 0x1e376c085141ab53,
    0x2748774cdf8eeb99, 0x34b0bcb5e19b48a8, 0x391c0cb3c5c95a63, 0x4ed8aa4ae3418acb, 0x5b9cca4f7763e373,
    0x682e6ff3d6b2b8a3, 0x748f82ee5defb2fc, 0x78a5636f43172f60, 0x84c87814a1f0ab72, 0x8cc702081a6439ec,
    0x90befffa23631e28, 0xa4506cebde82bde9, 0xbef9a3f7b2c67915, 0xc67178f2e372532b, 0xca273eceea26619c,
    0xd186b8c721c0c207, 0xeada7dd6cde0eb1e, 0xf57d4f7fee6ed178, 0x06f067aa72176fba, 0x0a637dc5a2c898a6,
    0x113f9804bef90dae, 0x1b710b35131c471b, 0x28db77f523047d84, 0x32caab7b40c72493, 0x3c9ebe0a15c9bebc,
    0x431d67c49c100d4c, 0x4cc5d4becb3e42b6, 0x597f299cfc657e2a, 0x5fcb6fab3ad6faec, 0x6c44198c4a475817]
SHA512_IV = [0x6a09e667f3bcc908, 0xbb67ae8584caa73b, 0x3c6ef372fe94f82b, 0xa54ff53a5f1d36f1,
             0x510e527fade682d1, 0x9b05688c2b3e6c1f, 0x1f83d9abfb41bd6b, 0x5be0cd19137e2179]


class Circuit:
    """Signals, constraints and witness operations of one circuit (see module docstring)."""

    def __init__(self, n_out: int, n_pub_in: int, n_prv_in: int, input_names=None, output_names=None):
        """input_names: [(name, size)] of the main's inputs in declaration order (sizes add
        up to n_pub_in + n_prv_in); written into the program so a caller can map an input
        object ({name: value | array}) onto the input signals, as circom's calculator does.
        output_names: [(name, size)] of the main's outputs (default: out[n_out])."""
        self.n_out, self.n_pub_in, self.n_prv_in = n_out, n_pub_in, n_prv_in
        self.input_names = list(input_names or [])
        if self.input_names and sum(k for _, k in self.input_names) != n_pub_in + n_prv_in:
            raise ValueError("input names do not cover the inputs")
        self.n_wires = 1 + n_out + n_pub_in + n_prv_in
        self.constraints = []          # (A, B, C)
        self.ops = []                  # (type, err, n, dst, A, B, C, extra) in creation order
        self.out_wires = list(range(1, 1 + n_out))
        self.in_base = 1 + n_out
        # signal names, circom's hierarchical "main.<component>.<signal>[i]" (write_sym)
        self.names = {}
        # further names, (name, wire or -1): signals equal to another signal's wire (a
        # component's inputs, an output passed on) or substituted away (-1), as circom's
        # .sym lists them (Circuit.declare)
        self.extra_names = []
        self._used = set()              # every name given so far (names stay unique)
        self._path = ["main"]
        self._seq = {}
        o = 1
        for name, k in list(output_names or [("out", n_out)]) + self.input_names:
            self._name(o, k, name)
            o += k

    # ---- allocation --------------------------------------------------------------
    def _name(self, base: int, n: int, sig: str, scalar: bool | None = None):
        prefix = ".".join(self._path)
        one = n == 1 if scalar is None else scalar
        for i in range(n):
            self.names[base + i] = nm = f"{prefix}.{sig}" if one else f"{prefix}.{sig}[{i}]"
            self._used.add(nm)

    def _next(self, kind: str) -> int:
        key = (len(self._path), ".".join(self._path), kind)
        k = self._seq.get(key, 0)
        self._seq[key] = k + 1
        return k

    @contextlib.contextmanager
    def component(self, kind: str, name: str | None = None):
        """Signals allocated inside are named <path>.<name>.<signal>. name: the component's
        name in its parent template (circom source); default <kind>[k], numbered per parent."""
        if name == "":          # the template's body inlined at the current level (a main)
            yield
            return
        if name is None:
            name = f"{kind}[{self._next(kind)}]"
        self._path.append(name)
        try:
            yield
        finally:
            self._path.pop()

    def alloc(self, n: int, name: str | None = None) -> int:
        base = self.n_wires
        self.n_wires += n
        if name is None:
            name = f"_s{self._next('_s')}"
            self._name(base, n, name, scalar=n == 1)
        else:
            self._name(base, n, name)
        return base

    def declare(self, sig: str, x):
        """circom's signal `sig` of the current component ("valueTally.nums": a signal of a
        sub-component) with value x: an LC or int, or a list of them for an array (nested
        for more dimensions). For the .sym only (no wire, constraint or operation): a
        value that is one wire still under an automatic name (_sN) takes the
        signal's name (e.g. a product the parent computed into this component's input, as
        circom names it); any other value adds a name, with the wire it equals (one wire,
        coefficient 1) or -1 (a constant or a combination: circom --O2 substitutes it)."""
        prefix = ".".join(self._path)

        def put(name, v):
            if name in self._used:      # e.g. a test main's output, named by the main itself
                return
            self._used.add(name)
            if isinstance(v, dict) and len(v) == 1:
                (wire, coef), = v.items()
                if wire and coef == 1:
                    cur = self.names.get(wire, "")
                    if cur.rsplit(".", 1)[-1].startswith("_s"):   # an automatic name: take it
                        self.names[wire] = name
                    elif cur != name:
                        self.extra_names.append((name, wire))
                    return
            self.extra_names.append((name, -1))

        def walk(name, v):
            if isinstance(v, (list, tuple)):
                for i, y in enumerate(v):
                    walk(f"{name}[{i}]", y)
            else:
                put(name, v)
        walk(f"{prefix}.{sig}", x)

    def write_sym(self) -> bytes:
        """circom's .sym text: one line per named signal, "label,wire,component,name": the
        allocated wires in wire order (every one has a name; wire 0 = the constant one has
        none, as in circom), then the declared further names (Circuit.declare), each with
        the wire it shares or -1."""
        comps, lines = {}, []
        entries = [(self.names[wire], wire) for wire in sorted(self.names)] + self.extra_names
        for label, (name, wire) in enumerate(entries, 1):
            comp = comps.setdefault(name.rsplit(".", 1)[0], len(comps))
            lines.append(f"{label},{wire},{comp},{name}\n")
        return "".join(lines).encode()

    def constrain(self, a, b, c):
        """A * B = C (A and B empty for a linear constraint)."""
        self.constraints.append((lc(a) if a is not None else {}, lc(b) if b is not None else {}, lc(c)))

    def _op(self, typ, dst, a=None, b=None, c=None, n=0, err=0, extra=None):
        self.ops.append((typ, err, n, dst, a, b, c, extra))

    # ---- signals -----------------------------------------------------------------
    def lin(self, x, dst: int | None = None, force: bool = False, name: str | None = None):
        """``s <== x`` for linear x: short combinations stay aliases (circom --O2
        substitutes them), longer ones become a signal with one linear constraint."""
        x = lc(x)
        if dst is None and not force and len(x) <= 2:
            return x
        s = self.alloc(1, name) if dst is None else dst
        self.constrain(None, None, sub(x, w(s)))
        self._op(OP_LIN, s, x)
        return w(s)

    def mul(self, a, b, c=0, dst: int | None = None, name: str | None = None):
        """``s <== a * b + c``."""
        a, b, c = lc(a), lc(b), lc(c)
        if is_const(a) or is_const(b):
            return self.lin(add(scale(b, const_value(a)) if is_const(a) else scale(a, const_value(b)), c), dst,
                            name=name)
        s = self.alloc(1, name) if dst is None else dst
        self.constrain(a, b, sub(w(s), c))
        self._op(OP_MUL, s, a, b, c)
        return w(s)

    def check_zero(self, x, err: int):
        """``x === 0`` (constraint plus the witness calculator's check)."""
        x = lc(x)
        if is_const(x):
            if const_value(x):
                raise ValueError("constant constraint fails")
            return
        self.constrain(None, None, x)
        self._op(OP_CHECK, 0, x, err=err)

    def check_quad(self, a, b, err: int):
        """``a * b === 0`` (constraint plus the witness calculator's check)."""
        a, b = lc(a), lc(b)
        self.constrain(a, b, 0)
        self._op(OP_CHECK, 0, a, b, err=err)

    def num2bits(self, x, n: int, err: int, name: str | None = None) -> list:
        """circomlib Num2Bits(n): n bit signals, LSB first."""
        with self.component("Num2Bits", name):
            base = self.alloc(n, "out")
            self.declare("in", lc(x))
        bits = [w(base + i) for i in range(n)]
        for b in bits:
            self.constrain(b, sub(b, 1), 0)
        self.constrain(None, None, sub(lc(x), add(*[scale(b, 1 << i) for i, b in enumerate(bits)])))
        self._op(OP_BITS, base, lc(x), n=n, err=err)
        return bits

    def is_zero(self, x, name: str | None = None) -> dict:
        """circomlib IsZero: inv <-- x != 0 ? 1/x : 0; out <== -x inv + 1; x out === 0."""
        x = lc(x)
        with self.component("IsZero", name):
            self.declare("in", x)
            inv = self.alloc(1, "inv")
            self._op(OP_INV, inv, x)
            out = self.mul(scale(x, -1), w(inv), 1, name="out")
        self.constrain(x, out, 0)
        return out

    def is_equal(self, a, b, name: str | None = None) -> dict:
        with self.component("IsEqual", name):
            self.declare("in", [lc(a), lc(b)])
            out = self.is_zero(sub(b, a), name="isz")
            self.declare("out", out)
            return out

    def less_than(self, a, b, n: int, err: int, name: str | None = None) -> dict:
        """circomlib LessThan(n): Num2Bits(n+1) of a + 2^n - b, out = 1 - bit n."""
        with self.component("LessThan", name):
            self.declare("in", [lc(a), lc(b)])
            bits = self.num2bits(add(a, 1 << n, scale(b, -1)), n + 1, err, name="n2b")
            self.declare("out", sub(1, bits[n]))
        return sub(1, bits[n])

    def quin(self, n: int, in_base: int, m: int, index, err_range: int, err_select: int,
             name: str | None = None) -> dict:
        """QuinSelector(n) (quinSelector.circom:11-42) over in[k] = wire in_base + k for
        k < m and 0 beyond: LessThan range check, then the IsZero/sum core as one op."""
        with self.component("QuinSelector", name):
            return self._quin(n, in_base, m, index, err_range, err_select)

    def _quin(self, n, in_base, m, index, err_range, err_select):
        bits = n.bit_length()          # log2(choices) + 1
        lt = self.less_than(index, n, bits, err_range, name="lessThan")
        self.check_zero(sub(lt, 1), err_select)
        index = lc(index)
        base = self.alloc(2 * n + m, "_block")
        prefix = ".".join(self._path)
        for i in range(n):
            self.names[base + i] = f"{prefix}.eqs[{i}].out"
            self.names[base + n + i] = f"{prefix}.eqs[{i}].inv"
        for i in range(m):
            self.names[base + 2 * n + i] = f"{prefix}.sums[{i}]"
        self._used.update(self.names[base + i] for i in range(2 * n + m))
        eq = lambda i: w(base + i)            # noqa: E731
        inv = lambda i: w(base + n + i)       # noqa: E731
        sums = lambda i: w(base + 2 * n + i)  # noqa: E731
        # circom's names of the inputs (in[k] = 0 past m), the output, eqs[i].in and the
        # sums past m (equal to sums[m - 1], as in[k] = 0 there)
        self.declare("in", [w(in_base + k) if k < m else 0 for k in range(n)])
        self.declare("index", index)
        self.declare("out", sums(m - 1) if m else 0)
        for i in range(n):
            self.declare(f"eqs[{i}].in", sub(i, index))
        for i in range(m, n):
            self.declare(f"sums[{i}]", sums(m - 1) if m else 0)
        for i in range(n):
            d = sub(i, index)
            self.constrain(d, inv(i), sub(1, eq(i)))
            self.constrain(d, eq(i), 0)
        for i in range(m):
            self.constrain(eq(i), w(in_base + i), sub(sums(i), sums(i - 1)) if i else sums(i))
        self._op(OP_QUIN, base, index, n=n, extra=(in_base, m))
        return sums(m - 1) if m else {}

    # ---- SHA-2 --------------------------------------------------------------------
    def sha_block(self, spec: dict, state_in, msg_bits: list, macro: int, extra) -> tuple:
        """Constraints of one SHA-2 compression (layout ``sha_block_layout``).
        state_in: 8 words of bit-LCs (LSB first) or ints; msg_bits: 16 words of bit-LCs.
        Returns (base wire, 8 output words of bit-LCs)."""
        L = sha_block_layout(spec)
        B = L["bits"]
        mask = (1 << B) - 1
        with self.component("Sha256compression" if B == 32 else "Sha512compression"):
            base = self.alloc(L["size"], "w")
        cur = [base]

        def take(k=1):
            s = cur[0]
            cur[0] += k
            return s

        def bitsof(word):
            return [lc((word >> i) & 1) for i in range(B)] if isinstance(word, int) else word

        def xor_word(x, r1, r2, r3, shr):
            x = bitsof(x)
            out = []
            for i in range(B):
                a, b = x[(i + r1) % B], x[(i + r2) % B]
                if shr and i + r3 >= B:        # XOR2: m = a b, a ^ b = a + b - 2m
                    m = take()
                    self.constrain(a, b, w(m))
                    out.append(add(a, b, scale(w(m), -2)))
                else:                           # XOR3 (circomlib Xor3)
                    c = x[(i + r3) % B] if not shr else x[i + r3]
                    mid, p = take(), take()
                    self.constrain(b, c, w(mid))
                    self.constrain(a, add(1, scale(b, -2), scale(c, -2), scale(w(mid), 4)), w(p))
                    out.append(add(w(p), b, c, scale(w(mid), -2)))
            return out

        def add_words(words, ncarry):
            """out bits (B) + ncarry carries = sum of words (bit-LC words or int constants)."""
            ob = take(B)
            cb = take(ncarry)
            outs = [w(ob + i) for i in range(B)] + [w(cb + j) for j in range(ncarry)]
            for o in outs:
                self.constrain(o, sub(o, 1), 0)
            total = {}
            for word in words:
                if isinstance(word, int):
                    total = add(total, word)
                else:
                    total = add(total, *[scale(bt, 1 << i) for i, bt in enumerate(word)])
            packed = add(*[scale(o, 1 << i) for i, o in enumerate(outs)])
            self.constrain(None, None, sub(packed, total))
            return outs[:B]

        K = SHA256_K if B == 32 else SHA512_K
        W = [msg_bits[t] for t in range(16)]
        for t in range(16, spec["rounds"]):
            s0 = xor_word(W[t - 15], *spec["s0"], True)
            s1 = xor_word(W[t - 2], *spec["s1"], True)
            W.append(add_words([s1, W[t - 7], s0, W[t - 16]], 2))
        a, b, c, d, e, f, g, h = [bitsof(x) for x in state_in]
        for t in range(spec["rounds"]):
            S1 = xor_word(e, *spec["S1"], False)
            q0 = take(B)
            ch = []
            for i in range(B):   # Ch = g + e (f - g)
                self.constrain(e[i], sub(f[i], g[i]), w(q0 + i))
                ch.append(add(w(q0 + i), g[i]))
            S0 = xor_word(a, *spec["S0"], False)
            mj = []
            q1 = take(2 * B)
            for i in range(B):   # Maj: mid = b c; q = a (b + c - 2 mid); maj = q + mid
                mid, q = w(q1 + 2 * i), w(q1 + 2 * i + 1)
                self.constrain(b[i], c[i], mid)
                self.constrain(a[i], add(b[i], c[i], scale(mid, -2)), q)
                mj.append(add(q, mid))
            t1 = [h, S1, ch, K[t] & mask, W[t]]
            na = add_words(t1 + [S0, mj], 3)
            ne = add_words([d] + t1, 3)
            h, g, f, e, d, c, b, a = g, f, e, ne, c, b, a, na
        V = [a, b, c, d, e, f, g, h]
        out = [add_words([state_in[j] if isinstance(state_in[j], int) else bitsof(state_in[j]), V[j]], 1)
               for j in range(8)]
        assert cur[0] == base + L["size"], (cur[0] - base, L["size"])
        self._op(macro, base, n=0, extra=extra)
        return base, out

    # ---- serialisation -----------------------------------------------------------
    def write_r1cs(self, wire_map: dict | None = None) -> bytes:
        """iden3 r1cs v1 (the file circom --r1cs writes; read by nzcb_plonk_setup).
        wire_map: {wire: new index} renumbering every wire but 0 (the same constraints in
        another wire order, e.g. the order of a .sym given to nzcb_wprog_remap)."""
        def le(x):
            return (x % R).to_bytes(32, "little")

        wm = (lambda k: k if k == 0 else wire_map[k]) if wire_map else (lambda k: k)  # noqa: E731

        hdr = struct.pack("<I", 32) + R.to_bytes(32, "little")
        hdr += struct.pack("<IIIIQI", self.n_wires, self.n_out, self.n_pub_in, self.n_prv_in, self.n_wires,
                           len(self.constraints))
        parts = []
        pack_i = struct.Struct("<I").pack
        for cons in self.constraints:
            for x in cons:
                parts.append(pack_i(len(x)))
                for k in sorted(x, key=wm):
                    parts.append(pack_i(wm(k)) + le(x[k]))
        body = b"".join(parts)
        labels = struct.pack(f"<{self.n_wires}Q", *range(self.n_wires))
        return _binfile(b"r1cs", 1, [(1, hdr), (2, body), (3, labels)])

    def write_program(self) -> bytes:
        """The witness program (format: csrc/wvm.hip header comment)."""
        consts, cidx = [], {}
        terms = []

        def put_lc(x):
            off = len(terms)
            for k in sorted(x):
                v = x[k]
                if v not in cidx:
                    cidx[v] = len(consts)
                    consts.append(v)
                terms.append((k, cidx[v]))
            return off, len(x)

        producer = {}
        level = []
        recs = []
        for order, (typ, err, n, dst, a, b, c, extra) in enumerate(self.ops):
            deps = []
            for x in (a, b, c):
                if x:
                    deps.extend(k for k in x if k)
            a_off, a_n = put_lc(a) if a else (0, 0)
            b_off, b_n = put_lc(b) if b else (0, 0)
            c_off, c_n = put_lc(c) if c else (0, 0)
            if typ == OP_QUIN:
                in_base, m = extra
                deps.extend(range(in_base, in_base + m))
                b_off, b_n = in_base, m
                width = 2 * n + m
            elif typ in (OP_SHA256, OP_SHA512):
                prev, msg = extra
                spec = SHA256_SPEC if typ == OP_SHA256 else SHA512_SPEC
                if prev is not None:
                    Lp = sha_block_layout(spec)
                    deps.extend(range(prev + Lp["final_base"], prev + Lp["size"]))
                deps.extend(range(msg, msg + 512))
                a_off, a_n = (prev if prev is not None else NO_WIRE), 0
                b_off, b_n = msg, 64
                width = sha_block_layout(spec)["size"]
            elif typ == OP_BITS:
                width = n
                c_off = order
            elif typ == OP_CHECK:
                width = 0
                c_off = order
            else:
                width = 1
            lv = 1 + max((producer.get(k, -1) for k in deps), default=-1)
            for k in range(dst, dst + width):
                producer[k] = lv
            level.append(lv)
            recs.append((typ | (err << 8) | (n << 16), dst, a_off, a_n, b_off, b_n, c_off, c_n))
        nlev = 1 + max(level, default=-1)
        # order: by level, scalar ops before macro ops inside a level
        idx = sorted(range(len(recs)), key=lambda i: (level[i], (recs[i][0] & 0xFF) in MACRO_OPS, i))
        starts, macro_starts = [], []
        pos = 0
        for lv in range(nlev):
            starts.append(pos)
            while pos < len(idx) and level[idx[pos]] == lv and (recs[idx[pos]][0] & 0xFF) not in MACRO_OPS:
                pos += 1
            macro_starts.append(pos)
            while pos < len(idx) and level[idx[pos]] == lv:
                pos += 1
        starts.append(pos)
        hdr = PROGRAM_MAGIC + struct.pack("<9I", PROGRAM_VERSION, self.n_wires, self.n_out, self.n_pub_in,
                                          self.n_prv_in, len(consts), len(terms), len(recs), nlev)
        out = [hdr, b"".join((v % R).to_bytes(32, "little") for v in consts)]
        out.append(struct.pack(f"<{2 * len(terms)}I", *[x for t in terms for x in t]))
        out.append(b"".join(struct.pack("<8I", *recs[i]) for i in idx))
        out.append(struct.pack(f"<{nlev + 1}I", *starts))
        out.append(struct.pack(f"<{nlev}I", *macro_starts))
        # input names: u32 count, then per input u32 name length, utf-8 name, u32 size
        out.append(struct.pack("<I", len(self.input_names)))
        for name, size in self.input_names:
            nb = name.encode()
            out.append(struct.pack("<I", len(nb)) + nb + struct.pack("<I", size))
        return b"".join(out)


def _binfile(magic: bytes, version: int, sections) -> bytes:
    out = [magic, struct.pack("<II", version, len(sections))]
    for sid, data in sections:
        out.append(struct.pack("<IQ", sid, len(data)))
        out.append(data)
    return b"".join(out)


def plonk_gate_count(c: Circuit) -> int:
    """Gates snarkjs ``plonk setup`` makes of the r1cs (oracle/r1cs.py process_constraints):
    one per public signal and constraint, plus (terms - 1) addition gates per linear
    combination with more than one non-constant term."""
    g = c.n_out + c.n_pub_in + len(c.constraints)
    for cons in c.constraints:
        for x in cons:
            k = sum(1 for wi in x if wi)
            if k > 1:
                g += k - 1
    return g
