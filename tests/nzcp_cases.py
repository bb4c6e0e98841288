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

import nzcb.nzcp  # noqa: F401  (input preparation: pass builders, CBOR codec)
from oracle import nzcp_circuit as nz
from oracle.bn254 import R_MOD

from nzcb.nzcp import (EXAMPLE_EXP, EXAMPLE_ISS, EXAMPLE_JTI, EXAMPLE_KID, EXAMPLE_NBF, LIVE_ISS,  # noqa: F401
                       LIVE_KID, Raw, claims, credential_subject, sig_structure)
from nzcb.nzcp import cbor_encode as cbor
from nzcb.nzcp import cbor_head as _head

DATA_1_20 = bytes(range(1, 21))   # test/nzcp.js:36


def to_be_signed(payload: bytes, kid: bytes = EXAMPLE_KID) -> bytes:
    return sig_structure(cbor({4: kid, 1: -7}), payload)


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
