"""R1CS -> PLONK circuit (snarkjs 0.4.12 ``plonk setup`` processConstraints), r1cs and
powers-of-tau file writers/readers, and a seeded satisfiable R1CS generator.

TEST INFRASTRUCTURE ONLY (see ``oracle/bn254.py`` header): the checker for
``nzcb_plonk_setup`` (csrc/synth.hip), never called by the product path.

PARITY UNPINNED against snarkjs: ``plonk_setup.js`` of snarkjs@0.4.12
(``/root/reference/yarn.lock:7279-7292``, run at ``/root/reference/Makefile:55,60``)
is [EXT] and absent, and the reference holds no r1cs, ptau or zkey files. This file
restates its processConstraints from the published algorithm:

* the nPublic = nOutputs + nPubInputs public signals get the first gates
  ``[s, 0, 0 | qm 0, ql 1, qr 0, qo 0, qc 0]``;
* each linear combination is read as (constant term k of wire 0, other terms); more
  than one other term is folded by reduceCoef: first half, second half, then a new
  signal ``so = c1 a + c2 b`` (gate ``[a, b, so | 0, -c1, -c2, 1, 0]`` plus the
  addition ``(a, b, c1, c2)``), numbered after the r1cs wires in creation order;
* ``(A)(B) = (C)`` becomes ``[A.s, B.s, C.s | A.c B.c, A.c B.k, A.k B.c, -C.c, A.k B.k - C.k]``;
* the domain is 2^(log2(nConstraints - 1) + 1), at least 2^3.

The processed circuit feeds ``oracle.plonk.setup`` (the rest of plonk_setup).
"""
from __future__ import annotations

import random
import struct

from . import bn254 as bn
from .binfmt import read_binfile, write_binfile
from .bn254 import P_MOD, R_MOD


def write_r1cs(n_wires: int, n_out: int, n_pub_in: int, n_prv_in: int, constraints) -> bytes:
    """iden3 r1cs v1. constraints: [(A, B, C)], each a list of (wire, coef) with coef
    in normal form (circom writes them reduced, little-endian)."""
    hdr = struct.pack("<I", 32) + bn.to_le(R_MOD)
    hdr += struct.pack("<IIIIQI", n_wires, n_out, n_pub_in, n_prv_in, n_wires, len(constraints))
    body = bytearray()
    for lcs in constraints:
        for lc in lcs:
            body += struct.pack("<I", len(lc))
            for w, c in lc:
                body += struct.pack("<I", w) + bn.to_le(c % R_MOD)
    labels = b"".join(struct.pack("<Q", i) for i in range(n_wires))
    return write_binfile(b"r1cs", 1, [(1, hdr), (2, bytes(body)), (3, labels)])


def read_r1cs(data: bytes) -> dict:
    _, sec = read_binfile(data, b"r1cs")
    (o, _), = sec[1]
    n8, = struct.unpack_from("<I", data, o)
    prime = bn.from_le(data[o + 4:o + 4 + n8])
    o += 4 + n8
    n_wires, n_out, n_pub_in, n_prv_in, n_labels, n_cons = struct.unpack_from("<IIIIQI", data, o)
    (o, _), = sec[2]
    cons = []
    for _ in range(n_cons):
        lcs = []
        for _ in range(3):
            nt, = struct.unpack_from("<I", data, o)
            o += 4
            lc = []
            for _ in range(nt):
                w, = struct.unpack_from("<I", data, o)
                lc.append((w, bn.from_le(data[o + 4:o + 4 + n8])))
                o += 4 + n8
            lcs.append(lc)
        cons.append(tuple(lcs))
    return {"prime": prime, "nWires": n_wires, "nOutputs": n_out, "nPubInputs": n_pub_in,
            "nPrvInputs": n_prv_in, "nLabels": n_labels, "constraints": cons}


def process_constraints(r1cs: dict) -> dict:
    """plonk_setup.js processConstraints + cirPower (see the module docstring)."""
    n_pub = r1cs["nOutputs"] + r1cs["nPubInputs"]
    nvars = [r1cs["nWires"]]
    gates, adds = [], []

    def reduce_coef(coefs):
        if not coefs:
            return 0, 0
        if len(coefs) == 1:
            return coefs[0]
        h = len(coefs) >> 1
        s1, c1 = reduce_coef(coefs[:h])
        s2, c2 = reduce_coef(coefs[h:])
        so = nvars[0]
        nvars[0] += 1
        gates.append([s1, s2, so, 0, -c1 % R_MOD, -c2 % R_MOD, 1, 0])
        adds.append((s1, s2, c1, c2))
        return so, 1

    def read_lc(lc):
        k = 0
        coefs = []
        for w, c in lc:
            if w == 0:
                k = c
            else:
                coefs.append((w, c))
        s, c = reduce_coef(coefs)
        return s, c, k

    for s in range(1, n_pub + 1):
        gates.append([s, 0, 0, 0, 1, 0, 0, 0])
    for A, B, C in r1cs["constraints"]:
        a = read_lc(A)
        b = read_lc(B)
        c = read_lc(C)
        gates.append([a[0], b[0], c[0], a[1] * b[1] % R_MOD, a[1] * b[2] % R_MOD, a[2] * b[1] % R_MOD,
                      -c[1] % R_MOD, (a[2] * b[2] - c[2]) % R_MOD])
    nc = len(gates)
    power = max((nc - 1).bit_length(), 3) if nc > 1 else 3
    return {"power": power, "constraints": gates, "nVars": nvars[0], "nPublic": n_pub,
            "nAdditions": len(adds), "additions": adds}


def extend_witness(circuit: dict, witness):
    """calculateAdditions: the witness of the addition signals, in creation order."""
    w = list(witness)
    for a, b, c1, c2 in circuit["additions"]:
        w.append((c1 * w[a] + c2 * w[b]) % R_MOD)
    return w


def write_ptau(tau: int, power: int, g2_points: int = 2) -> bytes:
    """snarkjs powers-of-tau layout, header and the two sections plonk setup reads:
    1 (n8, q, power, ceremonyPower), 2 tauG1 = [tau^i]G1 for i < 2^(power+1) - 1 and
    3 tauG2 = [tau^i]G2 (truncated to `g2_points`; the setup reads [tau]G2 only)."""
    s1 = struct.pack("<I", 32) + bn.to_le(P_MOD) + struct.pack("<II", power, power)
    g1 = bytearray()
    t = 1
    for _ in range((1 << (power + 1)) - 1):
        g1 += bn.g1_to_lem(bn.g1_mul(bn.G1_GEN, t))
        t = t * tau % R_MOD
    g2 = b"".join(bn.g2_to_lem(bn.g2_mul(bn.G2_GEN, pow(tau, i, R_MOD))) for i in range(g2_points))
    return write_binfile(b"ptau", 1, [(1, s1), (2, bytes(g1)), (3, g2)])


def random_r1cs(seed: int, n_out: int = 2, n_pub_in: int = 1, n_prv_in: int = 3, n_steps: int = 40):
    """A satisfiable r1cs in circom's wire order (one, outputs, public inputs, private
    inputs, intermediates) and its witness. Every step defines one new wire from earlier
    ones; the last n_out steps define the outputs. Linear combinations have 0-4 terms,
    constants, and sometimes an empty A or B (linear constraints)."""
    rng = random.Random(seed)
    n_in = n_pub_in + n_prv_in
    first_mid = 1 + n_out + n_in
    n_mid = n_steps - n_out
    n_wires = first_mid + n_mid
    w = [0] * n_wires
    w[0] = 1
    for i in range(1 + n_out, first_mid):
        w[i] = rng.randrange(R_MOD)
    known = list(range(1 + n_out, first_mid))
    used = set()
    targets = list(range(first_mid, n_wires)) + list(range(1, 1 + n_out))

    def lc(max_terms):
        terms = []
        for wire in rng.sample(known, min(len(known), rng.randrange(0, max_terms + 1))):
            terms.append((wire, rng.randrange(1, R_MOD)))
            used.add(wire)
        if rng.random() < 0.4:
            terms.append((0, rng.randrange(R_MOD)))
        rng.shuffle(terms)
        return terms

    def value(terms):
        return sum(c * w[s] for s, c in terms) % R_MOD

    cons = []
    for step, t in enumerate(targets):
        if step < n_in:  # use every input at least once
            A = [(known[step], rng.randrange(1, R_MOD))] + lc(2)
            used.add(known[step])
        else:
            A = lc(4) if rng.random() > 0.1 else []
        B = lc(3) if rng.random() > 0.1 else []
        rest = lc(2)
        ct = rng.randrange(1, R_MOD)
        # (A)(B) = ct * w_t + rest  ->  w_t = ((A)(B) - rest) / ct
        w[t] = (value(A) * value(B) - value(rest)) * bn.fr_inv(ct) % R_MOD
        C = rest + [(t, ct)]
        rng.shuffle(C)
        cons.append((A, B, C))
        known.append(t)
    return write_r1cs(n_wires, n_out, n_pub_in, n_prv_in, cons), w
