"""snarkjs 0.4 ``.zkey`` (PLONK) and ``.wtns`` binary formats.

TEST INFRASTRUCTURE ONLY (see ``oracle/bn254.py`` header).

Restates @iden3/binfileutils@0.0.10 sectioned files
(``/root/reference/yarn.lock:843-849``) and snarkjs 0.4.12 ``zkey_utils``
``readHeaderPlonk`` / ``wtns_utils`` layouts as summarised in SURVEY.md §8a
row a3:

* file  = magic[4] | u32 version | u32 nSections | sections
* section = u32 id | u64 size | payload
* zkey  section 1: u32 protocol (plonk = 2)
* zkey  section 2: n8q, q, n8r, r, nVars, nPublic, domainSize, nAdditions,
  nConstraints, k1 (LEM), k2 (LEM), Qm Ql Qr Qo Qc S1 S2 S3 (G1 LEM 64 B), X_2 (G2 LEM 128 B)
* zkey  section 3: additions, nAdditions x [u32 ai | u32 bi | ac LEM | bc LEM]
* zkey  sections 4/5/6: A/B/C wire maps, u32 x nConstraints
* zkey  sections 7..11: Qm Ql Qr Qo Qc, each n coefficients + 4n evaluations (LEM)
* zkey  section 12: sigma1..3, each n coefficients + 4n evaluations (LEM)
* zkey  section 13: Lagrange L_1..L_max(nPublic,1), each n + 4n (LEM)
* zkey  section 14: PTau, (n + 6) G1 LEM affine points
* wtns  (version 2): section 1 = u32 n8 | q | u32 nWitness; section 2 = witness (normal LE)
"""
from __future__ import annotations

import struct

from .bn254 import (P_MOD, R_MOD, from_le, from_lem, g1_from_lem, g1_to_lem, g2_from_lem,
                    g2_to_lem, to_le, to_lem)

PLONK_PROTOCOL_ID = 2


def write_binfile(magic: bytes, version: int, sections) -> bytes:
    out = bytearray(magic)
    out += struct.pack("<II", version, len(sections))
    for sid, payload in sections:
        out += struct.pack("<IQ", sid, len(payload))
        out += payload
    return bytes(out)


def read_binfile(data: bytes, magic: bytes):
    if data[:4] != magic:
        raise ValueError(f"{magic.decode()}: invalid file format")
    version, nsec = struct.unpack_from("<II", data, 4)
    off = 12
    sections = {}
    for _ in range(nsec):
        sid, size = struct.unpack_from("<IQ", data, off)
        off += 12
        sections.setdefault(sid, []).append((off, size))
        off += size
    return version, sections


def _fr_lem_array(vals):
    return b"".join(to_lem(v, R_MOD) for v in vals)


def write_zkey(zk: dict) -> bytes:
    """``zk`` holds normal-form ints; everything is converted to LEM here."""
    n = zk["domainSize"]
    s1 = struct.pack("<I", PLONK_PROTOCOL_ID)
    s2 = bytearray()
    s2 += struct.pack("<I", 32) + to_le(P_MOD)
    s2 += struct.pack("<I", 32) + to_le(R_MOD)
    s2 += struct.pack("<IIIII", zk["nVars"], zk["nPublic"], n, zk["nAdditions"], zk["nConstraints"])
    s2 += to_lem(zk["k1"], R_MOD) + to_lem(zk["k2"], R_MOD)
    for name in ("Qm", "Ql", "Qr", "Qo", "Qc", "S1", "S2", "S3"):
        s2 += g1_to_lem(zk[name])
    s2 += g2_to_lem(zk["X_2"])
    s3 = bytearray()
    for (ai, bi, ac, bc) in zk["additions"]:
        s3 += struct.pack("<II", ai, bi) + to_lem(ac, R_MOD) + to_lem(bc, R_MOD)
    s4 = struct.pack(f"<{len(zk['aMap'])}I", *zk["aMap"])
    s5 = struct.pack(f"<{len(zk['bMap'])}I", *zk["bMap"])
    s6 = struct.pack(f"<{len(zk['cMap'])}I", *zk["cMap"])
    sections = [(1, s1), (2, bytes(s2)), (3, bytes(s3)), (4, s4), (5, s5), (6, s6)]
    for sid, name in zip(range(7, 12), ("qm", "ql", "qr", "qo", "qc")):
        coefs, evals = zk[name]
        assert len(coefs) == n and len(evals) == 4 * n
        sections.append((sid, _fr_lem_array(coefs) + _fr_lem_array(evals)))
    s12 = b"".join(_fr_lem_array(c) + _fr_lem_array(e) for (c, e) in zk["sigma"])
    sections.append((12, s12))
    s13 = b"".join(_fr_lem_array(c) + _fr_lem_array(e) for (c, e) in zk["lagrange"])
    sections.append((13, s13))
    sections.append((14, b"".join(g1_to_lem(p) for p in zk["ptau"])))
    return write_binfile(b"zkey", 1, sections)


def _read_fr_lem(data, off, count):
    return [from_lem(data[off + 32 * i: off + 32 * i + 32], R_MOD) for i in range(count)]


def read_zkey(data: bytes) -> dict:
    _, sec = read_binfile(data, b"zkey")
    (o1, _), = sec[1]
    protocol, = struct.unpack_from("<I", data, o1)
    if protocol != PLONK_PROTOCOL_ID:
        raise ValueError("zkey file is not plonk")
    (o, _), = sec[2]
    zk = {"protocol": "plonk"}
    n8q, = struct.unpack_from("<I", data, o); o += 4
    zk["q"] = from_le(data[o:o + n8q]); o += n8q
    n8r, = struct.unpack_from("<I", data, o); o += 4
    zk["r"] = from_le(data[o:o + n8r]); o += n8r
    (zk["nVars"], zk["nPublic"], zk["domainSize"], zk["nAdditions"],
     zk["nConstraints"]) = struct.unpack_from("<IIIII", data, o); o += 20
    zk["k1"] = from_lem(data[o:o + 32], R_MOD); o += 32
    zk["k2"] = from_lem(data[o:o + 32], R_MOD); o += 32
    for name in ("Qm", "Ql", "Qr", "Qo", "Qc", "S1", "S2", "S3"):
        zk[name] = g1_from_lem(data[o:o + 64]); o += 64
    zk["X_2"] = g2_from_lem(data[o:o + 128]); o += 128
    n = zk["domainSize"]
    zk["power"] = n.bit_length() - 1
    (o, _), = sec[3]
    adds = []
    for i in range(zk["nAdditions"]):
        base = o + 72 * i
        ai, bi = struct.unpack_from("<II", data, base)
        ac = from_lem(data[base + 8:base + 40], R_MOD)
        bc = from_lem(data[base + 40:base + 72], R_MOD)
        adds.append((ai, bi, ac, bc))
    zk["additions"] = adds
    nc = zk["nConstraints"]
    for sid, name in ((4, "aMap"), (5, "bMap"), (6, "cMap")):
        (o, _), = sec[sid]
        zk[name] = list(struct.unpack_from(f"<{nc}I", data, o))
    for sid, name in zip(range(7, 12), ("qm", "ql", "qr", "qo", "qc")):
        (o, _), = sec[sid]
        zk[name] = (_read_fr_lem(data, o, n), _read_fr_lem(data, o + 32 * n, 4 * n))
    (o, _), = sec[12]
    zk["sigma"] = []
    for k in range(3):
        base = o + k * 5 * n * 32
        zk["sigma"].append((_read_fr_lem(data, base, n), _read_fr_lem(data, base + 32 * n, 4 * n)))
    (o, size), = sec[13]
    nl = size // (5 * n * 32)
    zk["lagrange"] = []
    for k in range(nl):
        base = o + k * 5 * n * 32
        zk["lagrange"].append((_read_fr_lem(data, base, n), _read_fr_lem(data, base + 32 * n, 4 * n)))
    (o, size), = sec[14]
    npts = size // 64
    zk["ptau"] = [g1_from_lem(data[o + 64 * i:o + 64 * i + 64]) for i in range(npts)]
    return zk


def write_wtns(witness) -> bytes:
    s1 = struct.pack("<I", 32) + to_le(R_MOD) + struct.pack("<I", len(witness))
    s2 = b"".join(to_le(v % R_MOD) for v in witness)
    return write_binfile(b"wtns", 2, [(1, s1), (2, s2)])


def read_wtns(data: bytes):
    _, sec = read_binfile(data, b"wtns")
    (o, _), = sec[1]
    n8, = struct.unpack_from("<I", data, o)
    q = from_le(data[o + 4:o + 4 + n8])
    nw, = struct.unpack_from("<I", data, o + 4 + n8)
    (o2, _), = sec[2]
    w = [from_le(data[o2 + n8 * i:o2 + n8 * i + n8]) for i in range(nw)]
    return {"q": q, "n8": n8, "nWitness": nw, "witness": w}
