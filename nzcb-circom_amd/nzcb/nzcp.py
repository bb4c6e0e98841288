"""NZ COVID Pass input preparation for the nzcp circuit.

Python mirror of ``nzcb-circom_amd/js/nzcp.js`` (the Node host's version), for the
bench and the Python API: pass URI -> COSE_Sign1 -> ToBeSigned bytes -> the circuit's
input signals, exactly as the reference tests build them
(``/root/reference/test/nzcp.js:33-42``, ``test/helpers/utils.js:2-89``,
``test/helpers/nzcp.js``):

* ``toBeSigned``: ``8 * maxLen`` bits, MSB first per byte, zero past the length
  (``bufferToBitArray(fitBytes(tbs, maxLen))``);
* ``toBeSignedLen``: the length in bytes;
* ``data``: the 20 pass-through bytes after ``evmRearrangeBytes`` (reversed byte
  order, reversed bits), as bits.

``input_signals`` packs them as the 32-byte LE field elements the GPU witness
kernel reads (include/nzcb.h ``nzcb_nzcp_witness``). ``sig_structure`` /
``claims`` build MoH-shaped passes (example or live key id and issuer) for tests
and the bench, which have no live pass (the reference reads those from env secrets).

Formats: base32 (RFC 4648, no padding), CBOR (RFC 7049, definite lengths),
COSE_Sign1 (RFC 8152, tag 18), CWT claims (RFC 8392: 1 iss, 4 exp, 5 nbf, 7 cti).
"""
from __future__ import annotations

import re

# circuits/nzcp_live.circom, nzcp_example.circom (NZCPPubIdentity parameters)
LIVE_TOBESIGNED_MAX = 351
EXAMPLE_TOBESIGNED_MAX = 314

EXAMPLE_PASS_URI = (  # /root/reference/test/nzcp.js:71 (MoH example pass)
    "NZCP:/1/2KCEVIQEIVVWK6JNGEASNICZAEP2KALYDZSGSZB2O5SWEOTOPJRXALTDN53GSZBRHEXGQZLBNR2GQLTOPICRUYMBTIFAIGTUKBA"
    "AUYTWMOSGQQDDN5XHIZLYOSBHQJTIOR2HA4Z2F4XXO53XFZ3TGLTPOJTS6MRQGE4C6Y3SMVSGK3TUNFQWY4ZPOYYXQKTIOR2HA4Z2F4X"
    "W46TDOAXGG33WNFSDCOJONBSWC3DUNAXG46RPMNXW45DFPB2HGL3WGFTXMZLSONUW63TFGEXDALRQMR2HS4DFQJ2FMZLSNFTGSYLCNRS"
    "UG4TFMRSW45DJMFWG6UDVMJWGSY2DN53GSZCQMFZXG4LDOJSWIZLOORUWC3CTOVRGUZLDOSRWSZ3JOZSW4TTBNVSWISTBMNVWUZTBNVU"
    "WY6KOMFWWKZ2TOBQXE4TPO5RWI33CNIYTSNRQFUYDILJRGYDVAYFE6VGU4MCDGK7DHLLYWHVPUS2YIDJOA6Y524TD3AZRM263WTY2BE4"
    "DPKIF27WKF3UDNNVSVWRDYIYVJ65IRJJJ6Z25M2DO4YZLBHWFQGVQR5ZLIWEQJOZTS3IQ7JTNCFDX")

EXAMPLE_KID = b"key-1"
LIVE_KID = b"z12Kf7UQ"
EXAMPLE_ISS = "did:web:nzcp.covid19.health.nz"
LIVE_ISS = "did:web:nzcp.identity.health.nz"
EXAMPLE_JTI = bytes.fromhex("60a4f54d4e304332be33ad78b1eafa4b")
EXAMPLE_NBF = 1635883530
EXAMPLE_EXP = 1951416330

_B32 = "ABCDEFGHIJKLMNOPQRSTUVWXYZ234567"


def base32_decode(s: str) -> bytes:
    out = bytearray()
    acc = bits = 0
    for ch in s:
        v = _B32.find(ch)
        if v < 0:
            raise ValueError("invalid base32 character")
        acc = ((acc << 5) | v) & 0xFFFF
        bits += 5
        if bits >= 8:
            bits -= 8
            out.append((acc >> bits) & 0xFF)
    return bytes(out)


class Tag:
    def __init__(self, tag: int, value):
        self.tag, self.value = tag, value


def cbor_decode(buf: bytes, off: int = 0):
    """Minimal CBOR decoder -> (value, next offset); maps keep key order."""
    ib = buf[off]
    off += 1
    major, info = ib >> 5, ib & 31
    if info < 24:
        arg = info
    elif info in (24, 25, 26, 27):
        n = 1 << (info - 24)
        arg = int.from_bytes(buf[off:off + n], "big")
        off += n
    else:
        raise ValueError("unsupported CBOR length encoding")
    if major == 0:
        return arg, off
    if major == 1:
        return -1 - arg, off
    if major == 2:
        return bytes(buf[off:off + arg]), off + arg
    if major == 3:
        return bytes(buf[off:off + arg]).decode(), off + arg
    if major == 4:
        a = []
        for _ in range(arg):
            v, off = cbor_decode(buf, off)
            a.append(v)
        return a, off
    if major == 5:
        m = {}
        for _ in range(arg):
            k, off = cbor_decode(buf, off)
            v, off = cbor_decode(buf, off)
            m[k] = v
        return m, off
    if major == 6:
        v, off = cbor_decode(buf, off)
        return Tag(arg, v), off
    simple = {20: False, 21: True, 22: None}
    if info in simple:
        return simple[info], off
    raise ValueError("unsupported CBOR item")


class Raw(bytes):
    """A pre-encoded CBOR item (lets tests build non-canonical encodings)."""


def cbor_head(major: int, n: int) -> bytes:
    if n < 24:
        return bytes([major << 5 | n])
    for info, size in ((24, 1), (25, 2), (26, 4), (27, 8)):
        if n < 1 << (8 * size):
            return bytes([major << 5 | info]) + n.to_bytes(size, "big")
    raise ValueError("CBOR argument too large")


def cbor_encode(x) -> bytes:
    """Minimal CBOR encoder (shortest heads, definite lengths, dict insertion order)."""
    if isinstance(x, Raw):
        return bytes(x)
    if isinstance(x, bool):
        return b"\xf5" if x else b"\xf4"
    if isinstance(x, int):
        return cbor_head(0, x) if x >= 0 else cbor_head(1, -1 - x)
    if isinstance(x, bytes):
        return cbor_head(2, len(x)) + x
    if isinstance(x, str):
        b = x.encode()
        return cbor_head(3, len(b)) + b
    if isinstance(x, list):
        return cbor_head(4, len(x)) + b"".join(cbor_encode(v) for v in x)
    if isinstance(x, dict):
        return cbor_head(5, len(x)) + b"".join(cbor_encode(k) + cbor_encode(v) for k, v in x.items())
    if isinstance(x, Tag):
        return cbor_head(6, x.tag) + cbor_encode(x.value)
    raise TypeError(type(x))


def decode_pass(pass_uri: str):
    """NZCP:/1/<base32> -> (protected header bytes, payload bytes, signature)."""
    m = re.fullmatch(r"NZCP:/(\d+)/([A-Z2-7]+)", pass_uri)
    if not m:
        raise ValueError("not an NZCP pass URI")
    cose, _ = cbor_decode(base32_decode(m.group(2)))
    if not isinstance(cose, Tag) or cose.tag != 18 or not isinstance(cose.value, list) or len(cose.value) != 4:
        raise ValueError("not a COSE_Sign1 structure")
    protected, _unprotected, payload, signature = cose.value
    return protected, payload, signature


def sig_structure(protected: bytes, payload: bytes) -> bytes:
    """COSE Sig_structure ["Signature1", body_protected, external_aad = h'', payload] (RFC 8152 §4.4)."""
    return cbor_encode(["Signature1", protected, b"", payload])


def to_be_signed(pass_uri: str) -> bytes:
    protected, payload, _ = decode_pass(pass_uri)
    return sig_structure(protected, payload)


def credential_subject(given="Jack", family="Sparrow", dob="1960-04-16", order=("givenName", "familyName", "dob")):
    vals = {"givenName": given, "familyName": family, "dob": dob}
    return {k: vals[k] for k in order}


def claims(iss=EXAMPLE_ISS, nbf=EXAMPLE_NBF, exp=EXAMPLE_EXP, subject=None, jti=EXAMPLE_JTI,
           order=(1, 5, 4, "vc", 7)) -> dict:
    """A MoH-shaped CWT claims map (the example pass's layout: the circuit's fixed
    credentialSubject offset, nzcptpl.circom:461, relies on it)."""
    vc = {
        "@context": ["https://www.w3.org/2018/credentials/v1", "https://nzcp.covid19.health.nz/contexts/v1"],
        "version": "1.0.0",
        "type": ["VerifiableCredential", "PublicCovidPass"],
        "credentialSubject": subject if subject is not None else credential_subject(),
    }
    vals = {1: iss, 5: nbf, 4: exp, "vc": vc, 7: jti}
    return {k: vals[k] for k in order}


def pass_tbs(live: bool = True, **claim_kw) -> bytes:
    """ToBeSigned of a MoH-shaped pass with the live (or example) key id and issuer."""
    claim_kw.setdefault("iss", LIVE_ISS if live else EXAMPLE_ISS)
    protected = cbor_encode({4: LIVE_KID if live else EXAMPLE_KID, 1: -7})
    return sig_structure(protected, cbor_encode(claims(**claim_kw)))


def bits_msb_first(bs: bytes) -> list:
    return [(b >> (7 - j)) & 1 for b in bs for j in range(8)]


def evm_rearrange(bs: bytes) -> bytes:
    """Reversed byte order, reversed bits within each byte (utils.js evmRearrangeBytes)."""
    return bytes(int(f"{b:08b}"[::-1], 2) for b in bs[::-1])


def circuit_input(tbs: bytes, data20: bytes = bytes(20), max_len: int = LIVE_TOBESIGNED_MAX) -> dict:
    """The input object of plonk.fullProve / calculateWitness (test/nzcp.js:41)."""
    if len(tbs) > max_len:
        raise ValueError(f"ToBeSigned is {len(tbs)} bytes, circuit takes {max_len}")
    if len(data20) != 20:
        raise ValueError("data must be 20 bytes")
    fitted = tbs + bytes(max_len - len(tbs))
    return {"toBeSigned": bits_msb_first(fitted), "toBeSignedLen": len(tbs),
            "data": bits_msb_first(evm_rearrange(data20))}


def input_signals(inp: dict) -> bytes:
    """Input object -> the main's input signals in declaration order (toBeSigned[],
    toBeSignedLen, data[]) as 32-byte LE field elements (nzcb_nzcp_witness layout)."""
    vals = list(inp["toBeSigned"]) + [inp["toBeSignedLen"]] + list(inp["data"])
    r = 21888242871839275222246405745257275088548364400416034343698204186575808495617
    return b"".join((int(v) % r).to_bytes(32, "little") for v in vals)
