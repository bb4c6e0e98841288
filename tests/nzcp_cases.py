"""NZ COVID Pass ToBeSigned builders and the nzcp witness parity cases.

Test infrastructure. The passes are COSE Sig_structure bytes laid out like the MoH
passes the reference tests use (test/nzcp.js:71 example pass; live passes come from
env secrets there, LIVE_PASS_URI_1..4, and are rebuilt here with the live key id and
issuer so the live circuit's offsets hold: claims map at byte 30, vcPos 80, credential
subject at 250, as test/nzcp.js:117,164,207 expect). Signatures are irrelevant: the
circuit hashes and parses the ToBeSigned only.
"""
from __future__ import annotations

import random

from oracle import nzcp_circuit as nz
from oracle.bn254 import R_MOD

EXAMPLE_JTI = bytes.fromhex("60a4f54d4e304332be33ad78b1eafa4b")
EXAMPLE_KID = b"key-1"
LIVE_KID = b"z12Kf7UQ"
EXAMPLE_ISS = "did:web:nzcp.covid19.health.nz"
LIVE_ISS = "did:web:nzcp.identity.health.nz"
EXAMPLE_NBF = 1635883530
EXAMPLE_EXP = 1951416330
DATA_1_20 = bytes(range(1, 21))   # test/nzcp.js:36


class Raw(bytes):
    """Pre-encoded CBOR item."""


def _head(major: int, n: int) -> bytes:
    if n < 24:
        return bytes([major << 5 | n])
    if n < 256:
        return bytes([major << 5 | 24, n])
    if n < 65536:
        return bytes([major << 5 | 25]) + n.to_bytes(2, "big")
    if n < 1 << 32:
        return bytes([major << 5 | 26]) + n.to_bytes(4, "big")
    return bytes([major << 5 | 27]) + n.to_bytes(8, "big")


def cbor(x) -> bytes:
    """Minimal CBOR encoder (RFC 7049 definite lengths); dicts keep insertion order."""
    if isinstance(x, Raw):
        return bytes(x)
    if isinstance(x, bool):
        return b"\xf5" if x else b"\xf4"
    if isinstance(x, int):
        return _head(0, x) if x >= 0 else _head(1, -1 - x)
    if isinstance(x, bytes):
        return _head(2, len(x)) + x
    if isinstance(x, str):
        b = x.encode()
        return _head(3, len(b)) + b
    if isinstance(x, list):
        return _head(4, len(x)) + b"".join(cbor(v) for v in x)
    if isinstance(x, dict):
        return _head(5, len(x)) + b"".join(cbor(k) + cbor(v) for k, v in x.items())
    raise TypeError(type(x))


def credential_subject(given="Jack", family="Sparrow", dob="1960-04-16", order=("givenName", "familyName", "dob")):
    vals = {"givenName": given, "familyName": family, "dob": dob}
    return {k: vals[k] for k in order}


def vc(subject: dict) -> dict:
    return {
        "@context": ["https://www.w3.org/2018/credentials/v1", "https://nzcp.covid19.health.nz/contexts/v1"],
        "version": "1.0.0",
        "type": ["VerifiableCredential", "PublicCovidPass"],
        "credentialSubject": subject,
    }


def claims(iss=EXAMPLE_ISS, nbf=EXAMPLE_NBF, exp=EXAMPLE_EXP, subject=None, jti=EXAMPLE_JTI, order=(1, 5, 4, "vc", 7)):
    vals = {1: iss, 5: nbf, 4: exp, "vc": vc(subject or credential_subject()), 7: jti}
    return {k: vals[k] for k in order}


def to_be_signed(payload: bytes, kid: bytes = EXAMPLE_KID) -> bytes:
    """COSE Sig_structure ["Signature1", protected, h'', payload] (RFC 8152 §4.4)."""
    protected = cbor({4: kid, 1: -7})
    return cbor(["Signature1", protected, b"", payload])


def example_tbs() -> bytes:
    return to_be_signed(cbor(claims()))


def live_tbs(**kw) -> bytes:
    kw.setdefault("iss", LIVE_ISS)
    return to_be_signed(cbor(claims(**kw)), kid=LIVE_KID)


# ---- cases --------------------------------------------------------------------------
def case(name, params, tbs: bytes, length=None, data=DATA_1_20, bit_overrides=None, data_fields=None):
    """A parity case: fitted ToBeSigned bytes plus optional raw field overrides."""
    mb = params["max_tbs_bytes"]
    fitted = (tbs + bytes(max(0, mb - len(tbs))))[:mb]
    return {
        "name": name, "params": dict(params), "tbs_hex": fitted.hex(),
        "len": str(len(tbs) if length is None else length),
        "data_hex": data.hex(), "bit_overrides": {str(k): str(v) for k, v in (bit_overrides or {}).items()},
        "data_fields": [str(v) for v in data_fields] if data_fields is not None else None,
    }


def case_signals(c):
    """(toBeSigned field ints, toBeSignedLen, data field ints) of a case."""
    params = c["params"]
    tbs = bytes.fromhex(c["tbs_hex"])
    bits, _, dbits = nz.circuit_input(tbs, bytes.fromhex(c["data_hex"]), params["max_tbs_bytes"])
    for k, v in c["bit_overrides"].items():
        bits[int(k)] = int(v)
    if c["data_fields"] is not None:
        dbits = [int(v) for v in c["data_fields"]]
    return bits, int(c["len"]), dbits


def case_input_bytes(c) -> bytes:
    bits, ln, data = case_signals(c)
    return b"".join(int(v).to_bytes(32, "little") for v in bits + [ln] + data)


def oracle_record(c) -> dict:
    bits, ln, data = case_signals(c)
    p = c["params"]
    w = nz.nzcp_pub_identity(bits, ln, data, p["is_live"], p["max_tbs_bytes"], p["max_array_len_vc"],
                             p["max_map_len_vc"])
    rec = {"status": w.status, "detail": w.detail}
    if w.status == nz.OK:
        rec.update({
            "exp": w.exp, "vc_pos": w.vc_pos, "given_len": nz.clamp32(w.given_len),
            "family_len": nz.clamp32(w.family_len), "dob_len": nz.clamp32(w.dob_len),
            "nullifier_len": nz.clamp32(w.nullifier_len), "tbs_sha256": w.tbs_sha256.hex(),
            "nullifier_sha512": w.nullifier_sha512.hex(), "nullifier": w.nullifier.hex(),
            "out": [str(v) for v in w.out],
        })
    return rec


def gpu_record_json(r: dict) -> dict:
    """GPU record (nzcb.nzcp_witness dict) in the oracle_record layout."""
    rec = {"status": r["status"], "detail": r["detail"]}
    if r["status"] == nz.OK:
        rec.update({k: r[k] for k in ("exp", "vc_pos", "given_len", "family_len", "dob_len", "nullifier_len")})
        rec.update({k: r[k].hex() for k in ("tbs_sha256", "nullifier_sha512", "nullifier")})
        rec["out"] = [str(v) for v in r["out"]]
    return rec


def all_cases(seed: int = 0x6E7A6370, n_mutations: int = 48):
    L, E = nz.LIVE_PARAMS, nz.EXAMPLE_PARAMS
    cs = [case("example pass, example circuit (test/nzcp.js:349)", E, example_tbs()),
          case("live-shaped pass, live circuit", L, live_tbs()),
          case("example pass in the live circuit (claims skip 30)", L, example_tbs()),
          case("zero data", L, live_tbs(), data=bytes(20)),
          case("all-ones data", L, live_tbs(), data=b"\xff" * 20)]
    names = [("Jo", "Bloggs", "1999-12-31"), ("Ana", "Te Whare", "2001-01-01"), ("X", "Y", "2"),
             ("", "Sparrow", "1960-04-16"), ("Jack", "", ""), ("Abcdefghijklmnopqrst", "Uvwxyzabcdefghijklmn", "1960-04-16"),
             ("A" * 21, "B" * 21, "1960-04-16"), ("A" * 22, "B", "1960-04-16"), ("A" * 23, "B", "1960-04-16"),
             ("A" * 24, "B", "1960-04-16"), ("A" * 30, "B", "1960-04-16"), ("A" * 32, "B", "C"),
             ("A" * 33, "B", "C"), ("A" * 31, "B" * 31, "C"), ("A" * 31, "B" * 32, "C"),
             ("José", "Ñúñez", "1960-04-16")]
    for g, f, d in names:
        cs.append(case(f"names {len(g.encode())}/{len(f.encode())}/{len(d.encode())}", L,
                       live_tbs(subject=credential_subject(g, f, d))))
    import itertools
    for perm in itertools.permutations(("givenName", "familyName", "dob")):
        cs.append(case(f"credentialSubject order {perm}", L, live_tbs(subject=credential_subject(order=perm))))
    dup = Raw(_head(5, 3) + cbor("givenName") + cbor("Jack") + cbor("givenName") + cbor("Jill")
              + cbor("dob") + cbor("1960-04-16"))
    cs.append(case("duplicate givenName key", L, live_tbs(subject=dup)))
    cs.append(case("credentialSubject key not a string", L, to_be_signed(
        cbor(claims(iss=LIVE_ISS, subject={"givenName": "Jack", "familyName": "Sparrow", 7: "1960-04-16"})),
        kid=LIVE_KID)))
    for exp_item, label in ((Raw(b"\x18\x2a"), "1-byte"), (Raw(b"\x19\x01\x02"), "2-byte"),
                            (Raw(b"\x17"), "immediate"), (Raw(b"\x1b" + (5).to_bytes(8, "big")), "8-byte")):
        cs.append(case(f"exp {label} encoding", L, live_tbs(exp=exp_item)))
    for order in ((1, 5, 4, 7, "vc"), ("vc", 1, 5, 4, 7), (4, 1, 5, "vc", 7), (1, 4, "vc", 5, 7)):
        cs.append(case(f"claims order {order}", L, live_tbs(order=order)))
    payload = cbor(claims(iss=LIVE_ISS))
    cs.append(case("claims map length 24 (DecodeUint23)", L, to_be_signed(Raw(b"\xb8\x18") + payload[1:], LIVE_KID)))
    cs.append(case("claims map length 3 (vc outside)", L, to_be_signed(bytes([0xa3]) + payload[1:], LIVE_KID)))
    cs.append(case("claims not a map", L, to_be_signed(bytes([0x85]) + payload[1:], LIVE_KID)))
    tbs = live_tbs()
    for ln in (0, 1, 30, 31, 200, len(tbs) - 1, 351, 352, 1000, R_MOD - 5, R_MOD - 200, 1 << 70):
        cs.append(case(f"toBeSignedLen {ln}", L, tbs, length=ln))
    for i, v in ((0, 2), (17, R_MOD - 1), (2807, 3), (100, R_MOD + 1), (5, (1 << 256) - 1)):
        cs.append(case(f"toBeSigned[{i}] = {v}", L, tbs, bit_overrides={i: v}))
    rng = random.Random(seed)
    for label, df in (("data non-bits small", [rng.randrange(4) for _ in range(160)]),
                      ("data random field", [rng.randrange(R_MOD) for _ in range(160)]),
                      ("data >= r", [R_MOD + rng.randrange(1 << 250) for _ in range(160)])):
        cs.append(case(label, L, tbs, data_fields=df))
    long_subj = credential_subject("A" * 20, "B" * 20, "C" * 14)
    long_tbs = live_tbs(subject=long_subj)
    cs.append(case(f"long pass ({len(long_tbs)} B)", L, long_tbs))
    pad = 351 - len(long_tbs)
    at_max = live_tbs(subject=credential_subject("A" * 20, "B" * 20, "C" * (14 + pad)))
    cs.append(case(f"pass at MaxToBeSignedBytes ({len(at_max)} B)", L, at_max))
    over = live_tbs(subject=credential_subject("A" * 20, "B" * 20, "C" * (15 + pad)))
    cs.append(case(f"pass over MaxToBeSignedBytes ({len(over)} B, fitted)", L, over, length=len(over)))
    for k in range(n_mutations):
        b = bytearray(tbs)
        for _ in range(1 + k % 3):
            b[rng.randrange(27, len(b))] = rng.randrange(256)
        cs.append(case(f"mutation {k}", L, bytes(b), data=bytes(rng.randrange(256) for _ in range(20))))
    for k in range(8):
        cs.append(case(f"random bytes {k}", L, bytes(rng.randrange(256) for _ in range(351))))
    return cs
