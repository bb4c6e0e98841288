"""CPU evaluation of a witness program (the format written by
``nzcb.circuit.Circuit.write_program``, run on the GPU by ``csrc/wvm.hip``).

TEST INFRASTRUCTURE ONLY (see ``oracle/bn254.py`` header): the checker for the GPU
witness VM; only ``tests/`` and ``__graft_entry__.smoke()`` may use it.

It restates the witness rules the program encodes, one operation at a time, in plain
Python integers: circomlib Num2Bits (``out[i] <-- (in >> i) & 1``), IsZero
(``inv <-- in != 0 ? 1/in : 0``), QuinSelector's IsZero/sum core
(/root/reference/circuits/quinSelector.circom:27-38), and SHA-2 compressions
(FIPS 180-4) emitted signal by signal in the layout documented at
``nzcb.circuit.sha_block_layout``. A failing BITS/CHECK records (creation order, err);
the lowest order wins. Independent of the GPU code; the r1cs check
(``r1cs_unsatisfied``) makes it independent of the program too: a witness that
satisfies every constraint and has the right public outputs is the circuit's witness.
"""
from __future__ import annotations

import struct

from .bn254 import R_MOD as R

OP_LIN, OP_MUL, OP_INV, OP_BITS, OP_CHECK, OP_QUIN, OP_SHA256, OP_SHA512 = range(8)
NO_WIRE = 0xFFFFFFFF


def parse(prog: bytes) -> dict:
    if prog[:4] != b"nzwp":
        raise ValueError("not a witness program")
    ver, n_wires, n_out, n_pub, n_prv, n_consts, n_terms, n_ops, n_lev = struct.unpack_from("<9I", prog, 4)
    o = 40
    consts = [int.from_bytes(prog[o + 32 * i:o + 32 * i + 32], "little") for i in range(n_consts)]
    o += 32 * n_consts
    t = struct.unpack_from(f"<{2 * n_terms}I", prog, o)
    terms = [(t[2 * i], t[2 * i + 1]) for i in range(n_terms)]
    o += 8 * n_terms
    ops = [struct.unpack_from("<8I", prog, o + 32 * i) for i in range(n_ops)]
    o += 32 * n_ops
    starts = struct.unpack_from(f"<{n_lev + 1}I", prog, o)
    if ver != 2:
        raise ValueError("unsupported witness program version")
    o += 4 * (n_lev + 1) + 4 * n_lev
    (n_names,) = struct.unpack_from("<I", prog, o)
    o += 4
    for _ in range(n_names):
        (ln,) = struct.unpack_from("<I", prog, o)
        o += 8 + ln
    wmap = None
    if o != len(prog):     # nzcb_wprog_remap's wire map: output wire t = program wire map[t]
        if prog[o:o + 4] != b"wmap":
            raise ValueError("witness program: trailing bytes")
        (T,) = struct.unpack_from("<I", prog, o + 4)
        wmap = list(struct.unpack_from(f"<{T}I", prog, o + 8))
    return dict(n_wires=n_wires, n_out=n_out, n_pub=n_pub, n_prv=n_prv, consts=consts, terms=terms, ops=ops,
                levels=starts, wmap=wmap)


def _lc(p, wit, off, n):
    s = 0
    terms, consts = p["terms"], p["consts"]
    for i in range(off, off + n):
        wire, ci = terms[i]
        s += consts[ci] * wit[wire]
    return s % R


_INV_CACHE = {}


def _inv(x):
    """1/x mod r (0 for 0); the IsZero inverses of small integers +-d repeat, so cache them."""
    if not x:
        return 0
    v = _INV_CACHE.get(x)
    if v is None:
        v = pow(x, R - 2, R)
        if x < 1 << 16 or R - x < 1 << 16:
            _INV_CACHE[x] = v
    return v


# ---- SHA-2 (FIPS 180-4), values in the circuit layout --------------------------------
def _sha_constants(bits):
    from nzcb import circuit as C   # round constants / IVs only (FIPS 180-4 tables)
    if bits == 32:
        return C.SHA256_K, C.SHA256_IV, (2, 13, 22), (6, 11, 25), (7, 18, 3), (17, 19, 10), 64
    return C.SHA512_K, C.SHA512_IV, (28, 34, 39), (14, 18, 41), (1, 8, 7), (19, 61, 6), 80


def sha_block_values(bits: int, state: list, msg_words: list) -> list:
    """Every signal value of one compression, in layout order."""
    K, _, S0, S1, s0, s1, rounds = _sha_constants(bits)
    mask = (1 << bits) - 1
    out = []

    def bit(x, i):
        return (x >> i) & 1

    def xor_sig(x, r1, r2, r3, shr):
        val = 0
        for i in range(bits):
            a, b = bit(x, (i + r1) % bits), bit(x, (i + r2) % bits)
            if shr and i + r3 >= bits:
                out.append(a * b)
                val |= (a ^ b) << i
            else:
                c = bit(x, i + r3) if shr else bit(x, (i + r3) % bits)
                mid = b * c
                out.append(mid)
                out.append(a * (1 - 2 * b - 2 * c + 4 * mid) % R)
                val |= (a ^ b ^ c) << i
        return val

    def add_sig(total, ncarry):
        for i in range(bits + ncarry):
            out.append((total >> i) & 1)
        return total & mask

    W = list(msg_words)
    for t in range(16, rounds):
        x0 = xor_sig(W[t - 15], *s0, True)
        x1 = xor_sig(W[t - 2], *s1, True)
        W.append(add_sig(x1 + W[t - 7] + x0 + W[t - 16], 2))
    a, b, c, d, e, f, g, h = state
    for t in range(rounds):
        S1v = xor_sig(e, *S1, False)
        ch = 0
        for i in range(bits):
            ei, fi, gi = bit(e, i), bit(f, i), bit(g, i)
            out.append(ei * (fi - gi) % R)
            ch |= ((ei & fi) ^ ((1 - ei) & gi)) << i
        S0v = xor_sig(a, *S0, False)
        mj = 0
        for i in range(bits):
            ai, bi, ci = bit(a, i), bit(b, i), bit(c, i)
            mid = bi * ci
            out.append(mid)
            out.append(ai * (bi + ci - 2 * mid))
            mj |= ((ai & bi) ^ (ai & ci) ^ (bi & ci)) << i
        t1 = h + S1v + ch + K[t] + W[t]
        na = add_sig(t1 + S0v + mj, 3)
        ne = add_sig(d + t1, 3)
        h, g, f, e, d, c, b, a = g, f, e, ne, c, b, a, na
    V = [a, b, c, d, e, f, g, h]
    for j in range(8):
        add_sig(state[j] + V[j], 1)
    return out


def _sha_final_words(bits, wit, base, size):
    fb = base + size - 8 * (bits + 1)
    return [sum((wit[fb + j * (bits + 1) + i] & 1) << i for i in range(bits)) for j in range(8)]


def _msg_words(wit, byte_base, nbytes, bits):
    # a message wire that is not a bit (only in a witness that already failed a check)
    # contributes its lowest bit, as the GPU VM reads it
    data = bytes(sum((wit[byte_base + 8 * k + j] & 1) << j for j in range(8)) for k in range(nbytes))
    nb = bits // 8
    return [int.from_bytes(data[nb * t:nb * t + nb], "big") for t in range(len(data) // nb)]


def _layout_size(bits):
    from nzcb import circuit as C
    return C.sha_block_layout(C.SHA256_SPEC if bits == 32 else C.SHA512_SPEC)["size"]


def evaluate(prog: bytes, inputs: list) -> tuple:
    """inputs: the main's input signals (ints) in declaration order. Returns (witness
    list of n_wires ints, failure (order, err) or None)."""
    p = parse(prog)
    wit = [0] * p["n_wires"]
    wit[0] = 1
    base = 1 + p["n_out"]
    if len(inputs) != p["n_pub"] + p["n_prv"]:
        raise ValueError("wrong number of input signals")
    for i, v in enumerate(inputs):
        wit[base + i] = v % R
    fail = None

    def failed(order, err):
        nonlocal fail
        if fail is None or order < fail[0]:
            fail = (order, err)

    for op in p["ops"]:
        code, dst, a_off, a_n, b_off, b_n, c_off, c_n = op
        typ, err, n = code & 0xFF, (code >> 8) & 0xFF, code >> 16
        if typ == OP_LIN:
            wit[dst] = _lc(p, wit, a_off, a_n)
        elif typ == OP_MUL:
            wit[dst] = (_lc(p, wit, a_off, a_n) * _lc(p, wit, b_off, b_n) + _lc(p, wit, c_off, c_n)) % R
        elif typ == OP_INV:
            wit[dst] = _inv(_lc(p, wit, a_off, a_n))
        elif typ == OP_BITS:
            x = _lc(p, wit, a_off, a_n)
            for i in range(n):
                wit[dst + i] = (x >> i) & 1
            if x >> n:
                failed(c_off, err)
        elif typ == OP_CHECK:
            x = _lc(p, wit, a_off, a_n)
            if b_n:
                x = x * _lc(p, wit, b_off, b_n) % R
            if x:
                failed(c_off, err)
        elif typ == OP_QUIN:
            idx = _lc(p, wit, a_off, a_n)
            for i in range(n):
                d = (i - idx) % R
                wit[dst + i] = 1 if d == 0 else 0
                wit[dst + n + i] = _inv(d)
            s = 0
            for i in range(b_n):
                s = (s + wit[dst + i] * wit[b_off + i]) % R
                wit[dst + 2 * n + i] = s
        elif typ in (OP_SHA256, OP_SHA512):
            bits = 32 if typ == OP_SHA256 else 64
            if a_off == NO_WIRE:
                state = list(_sha_constants(bits)[1])
            else:
                state = _sha_final_words(bits, wit, a_off, _layout_size(bits))
            words = _msg_words(wit, b_off, 64, bits)
            if typ == OP_SHA512:      # one block of a 64-byte message: constant padding
                words += [1 << 63] + [0] * 6 + [512]
            vals = sha_block_values(bits, state, words)
            wit[dst:dst + len(vals)] = vals
        else:
            raise ValueError(f"unknown op {typ}")
    if p["wmap"] is not None:
        wit = [wit[k] for k in p["wmap"]]
    return wit, fail


def r1cs_unsatisfied(r1cs: dict, wit: list, limit: int = 5) -> list:
    """Indices of constraints A*B != C (oracle.r1cs.read_r1cs layout), at most `limit`."""
    bad = []
    for k, (A, B, C) in enumerate(r1cs["constraints"]):
        a = sum(c * wit[i] for i, c in A) % R
        b = sum(c * wit[i] for i, c in B) % R
        cc = sum(c * wit[i] for i, c in C) % R
        if (a * b - cc) % R:
            bad.append(k)
            if len(bad) >= limit:
                break
    return bad
