"""CPU restatement of the nzcp circuit's witness semantics (``NZCPPubIdentity``).

TEST INFRASTRUCTURE ONLY (see ``oracle/bn254.py`` header): the checker for the
HIP witness kernel ``nzcb-circom_amd/csrc/nzcp.hip``; only ``tests/`` and
``__graft_entry__.smoke()`` may import it.

What it restates: the values the circom witness
calculator assigns to the circuit's *semantic* signals and its outputs, and
which inputs make it throw, for

    NZCPPubIdentity(IsLive, MaxToBeSignedBytes, MaxCborArrayLenVC, MaxCborMapLenVC, ...)
        /root/reference/circuits/nzcptpl.circom:444-655
    cbortpl.circom:26-503 (GetType, GetX, GetV, DecodeUint23, DecodeUint, ReadType,
        SkipValueScalar, SkipValue, StringEquals, ReadStringLength, ReadMapLength, CopyString)
    quinSelector.circom:11-42, log2.circom:5-12

Every gadget follows its template's arithmetic exactly, including the field
wrap-around of circomlib ``LessThan(n)`` (``Num2Bits(n+1)`` of ``a + 2^n - b``:
the witness calculator rejects operands whose difference leaves
``[-2^n, 2^n)``), the ``QuinSelector`` range check (an index in
``[choices - 2^bits, 0)`` selects 0, an index ``>= choices`` throws), and the
"every branch is evaluated" behaviour of ``DecodeUint`` / ``StringEquals`` /
``CopyString`` (their reads are range-checked even when their result is
multiplied by 0). ``===`` constraints are checked while the witness is
computed (the reference's own tests expect rejections from pure constraints,
e.g. ``test/quinSelector.js:63-86``, ``test/cbor.js:128-141``).

Values are signed Python ints: all positions/lengths in this circuit stay far
below 2^64 before a range check consumes them, and a negative int ``-m``
stands for the field element ``r - m``.

Pinning: ``tests/test_nzcp_oracle.py`` checks every gadget against the
reference's gadget KATs (``test/cbor.js``, ``test/quinSelector.js``) and the
whole circuit against the reference test's decode of the example pass
(``test/nzcp.js:33-69``, ``test/utils.js:16-20``: SHA-256 of the ToBeSigned,
vcPos 76 / credential subject 246/247, the nullifier ``Jack,Sparrow,1960-04-16``).
SHA-256 (``Sha256Var(3)``) and SHA-512 (``Sha512(512)``) come from external
circom libraries that are not on disk; they are restated as the
standard FIPS 180-4 functions, which is what the reference test decodes the
outputs against. One corner is **unpinned**: the reference inputs always
zero-fill the bits past ``toBeSignedLen`` (``fitBytes``); what ``Sha256Var``
does with non-zero bits there, or with a negative length, is unknown, so the
restatement hashes the first ``toBeSignedLen`` bytes and rejects negative
lengths with ``ERR_UNPINNED``.
"""
from __future__ import annotations

import hashlib

from .bn254 import R_MOD

# error codes, shared with include/nzcb.h (NZCB_NZCP_*)
OK = 0
ERR_BIT = 1          # toBeSigned[i] * (toBeSigned[i] - 1) === 0     nzcptpl.circom:493-496
ERR_LEN = 2          # lteMaxToBeSignedBytes.out === 1                 nzcptpl.circom:500-505
ERR_RANGE = 3        # LessThan / Num2Bits operand out of its bit range (circomlib comparators)
ERR_SELECT = 4       # QuinSelector: lessThan.out === 1 (index >= choices)  quinSelector.circom:20-25
ERR_NOT_MAP = 5      # ReadMapLength: type === MAJOR_TYPE_MAP          cbortpl.circom:449
ERR_UINT23 = 6       # DecodeUint23: x < 24                            cbortpl.circom:109-113
ERR_NOT_STRING = 7   # ReadStringLength: type === MAJOR_TYPE_STRING    cbortpl.circom:417
ERR_UNPINNED = 8     # negative toBeSignedLen (Sha256Var behaviour not on disk)

ERR_NAMES = {
    OK: "ok", ERR_BIT: "toBeSigned bit check", ERR_LEN: "toBeSignedLen > MaxToBeSignedBytes",
    ERR_RANGE: "LessThan operands out of range", ERR_SELECT: "QuinSelector index out of range",
    ERR_NOT_MAP: "CBOR type is not a map", ERR_UINT23: "CBOR map length > 23",
    ERR_NOT_STRING: "CBOR type is not a string", ERR_UNPINNED: "negative toBeSignedLen (unpinned)",
}

MAJOR_INT, MAJOR_STRING, MAJOR_ARRAY, MAJOR_MAP = 0, 3, 4, 5
COMMA = 44
CREDENTIAL_SUBJECT_VC_OFFSET = 171      # nzcptpl.circom:461
CREDENTIAL_SUBJECT_MAP_LEN = 3          # nzcptpl.circom:462
NULLIFIER_BYTES = 64                    # nzcptpl.circom:466
DATA_BITS = 160                         # nzcptpl.circom:474
CHUNK_BITS = 248
# NZCPPubIdentity parameters of the two mains (circuits/nzcp_example.circom, nzcp_live.circom)
EXAMPLE_PARAMS = dict(is_live=0, max_tbs_bytes=314, max_array_len_vc=0, max_map_len_vc=4)
LIVE_PARAMS = dict(is_live=1, max_tbs_bytes=351, max_array_len_vc=0, max_map_len_vc=4)

VC = b"vc"
GIVEN_NAME = b"givenName"
FAMILY_NAME = b"familyName"
DOB = b"dob"


class CircuitError(Exception):
    def __init__(self, code: int, detail: int = 0):
        super().__init__(f"{ERR_NAMES[code]} (detail {detail})")
        self.code = code
        self.detail = detail


def log2(x: int) -> int:
    """log2.circom:5-12 (floor log2, log2(0) = -1)."""
    z = -1
    while x:
        z += 1
        x //= 2
    return z


def clamp32(x: int) -> int:
    return max(-(1 << 31), min((1 << 31) - 1, x))


# ---- circomlib comparators / quinSelector ------------------------------------
def less_than(n: int, a: int, b: int) -> int:
    """circomlib LessThan(n): Num2Bits(n+1) of a + 2^n - b, out = 1 - bit n."""
    t = a + (1 << n) - b
    if not 0 <= t < (1 << (n + 1)):
        raise CircuitError(ERR_RANGE, clamp32(a))
    return 1 if t < (1 << n) else 0


def quin_selector(arr, index: int) -> int:
    """quinSelector.circom:11-42."""
    choices = len(arr)
    if choices == 0:
        return 0
    bits = log2(choices) + 1
    t = index + (1 << bits) - choices
    if not 0 <= t < (1 << bits):          # Num2Bits(bits+1) fails, or lessThan.out === 1 fails
        raise CircuitError(ERR_SELECT, clamp32(index))
    return arr[index] if 0 <= index < choices else 0


def num2bits_check(n: int, v: int) -> None:
    if not 0 <= v < (1 << n):
        raise CircuitError(ERR_RANGE, clamp32(v))


# ---- cbortpl.circom ----------------------------------------------------------
def get_type(v: int) -> int:
    """GetType (cbortpl.circom:26-52): v >> 5 of a byte."""
    num2bits_check(8, v)
    return v >> 5


def get_x(v: int) -> int:
    """GetX (cbortpl.circom:54-73): v & 31 of a byte."""
    num2bits_check(8, v)
    return v & 31


def get_v(bs, pos: int) -> int:
    """GetV (cbortpl.circom:75-91)."""
    return quin_selector(bs, pos)


def decode_uint23(v: int) -> int:
    """DecodeUint23 (cbortpl.circom:93-114)."""
    x = get_x(v)
    if less_than(8, x, 24) != 1:
        raise CircuitError(ERR_UINT23, x)
    return x


def decode_uint(bs, pos: int, v: int):
    """DecodeUint (cbortpl.circom:116-237) -> (value, nextPos)."""
    x = get_x(v)
    c23 = less_than(8, x, 24)
    c24, c25, c26 = int(x == 24), int(x == 25), int(x == 26)
    v24 = get_v(bs, c24 * pos)
    v1_25 = get_v(bs, c25 * pos)
    v2_25 = get_v(bs, c25 * (pos + 1))
    v1_26 = get_v(bs, c26 * pos)
    v2_26 = get_v(bs, c26 * (pos + 1))
    v3_26 = get_v(bs, c26 * (pos + 2))
    v4_26 = get_v(bs, c26 * (pos + 3))
    value = (c23 * x + c24 * v24 + c25 * (v1_25 * 256 + v2_25)
             + c26 * (v1_26 * 16777216 + v2_26 * 65536 + v3_26 * 256 + v4_26))
    next_pos = c23 * pos + c24 * (pos + 1) + c25 * (pos + 2) + c26 * (pos + 4)
    return value, next_pos


def read_type(bs, pos: int):
    """ReadType (cbortpl.circom:239-262) -> (nextPos, type, v)."""
    v = get_v(bs, pos)
    return pos + 1, get_type(v), v


def skip_value_scalar(bs, pos: int) -> int:
    """SkipValueScalar (cbortpl.circom:264-297)."""
    nt, t, v = read_type(bs, pos)
    value, np_ = decode_uint(bs, nt, v)
    return int(t == MAJOR_INT) * np_ + int(t == MAJOR_STRING) * (np_ + value)


def skip_value(bs, pos: int, max_array_len: int) -> int:
    """SkipValue (cbortpl.circom:300-360)."""
    nt, t, v = read_type(bs, pos)
    value, np_ = decode_uint(bs, nt, v)
    is_int, is_str, is_arr = int(t == MAJOR_INT), int(t == MAJOR_STRING), int(t == MAJOR_ARRAY)
    nexts = []
    for i in range(max_array_len):
        lt = less_than(log2(max_array_len) + 1, i, is_arr * value)
        consider = is_arr * lt
        p = (np_ if i == 0 else nexts[i - 1]) * consider
        nexts.append(skip_value_scalar(bs, p))
    qs = quin_selector(nexts, is_arr * (value - 1))
    return is_int * np_ + is_str * (np_ + value) + is_arr * qs


def string_equals(bs, pos: int, length: int, const: bytes) -> int:
    """StringEquals (cbortpl.circom:362-400)."""
    s = int(length == len(const))
    for i, c in enumerate(const):
        s += int(c == get_v(bs, pos + i))
    return int(len(const) + 1 - s == 0)


def read_string_length(bs, pos: int):
    """ReadStringLength (cbortpl.circom:402-425) -> (len, nextPos); nextPos is pos + 1."""
    nt, t, v = read_type(bs, pos)
    if t != MAJOR_STRING:
        raise CircuitError(ERR_NOT_STRING, clamp32(pos))
    value, _ = decode_uint(bs, nt, v)
    return value, nt


def read_map_length(bs, pos: int):
    """ReadMapLength (cbortpl.circom:427-451) -> (len, nextPos)."""
    nt, t, v = read_type(bs, pos)
    if t != MAJOR_MAP:
        raise CircuitError(ERR_NOT_MAP, clamp32(pos))
    return decode_uint23(v), nt


def copy_string(bs, pos: int, max_len: int):
    """CopyString (cbortpl.circom:453-503) -> (outbytes, nextPos, len)."""
    slen, np_ = read_string_length(bs, pos)
    bits = log2(max_len) + 1
    out = []
    for i in range(max_len):
        b = get_v(bs, np_ + i)
        out.append(b * less_than(bits, i, slen))
    return out, np_ + slen, slen


# ---- nzcptpl.circom ----------------------------------------------------------
def find_cwt_claims(bs, pos: int, map_len: int, max_array_len: int, max_map_len: int):
    """FindCWTClaims (nzcptpl.circom:28-145) -> (vcPos, exp)."""
    vc_pos = 0
    exp_pos = 0
    p = pos
    for k in range(max_map_len):
        nt, t, v = read_type(bs, p)
        value, np_ = decode_uint(bs, nt, v)
        is_str, is_int = int(t == MAJOR_STRING), int(t == MAJOR_INT)
        p_next = skip_value(bs, np_ + value * is_str, max_array_len)
        needle = string_equals(bs, np_, value, VC)
        is4 = int(value == 4)
        within = less_than(8, k, map_len)
        vc_pos += is_str * needle * within * (np_ + value)
        exp_pos += is_int * is4 * within * np_
        p = p_next
    nt, t, v = read_type(bs, exp_pos)
    exp, _ = decode_uint(bs, nt, v)
    return vc_pos, exp


CREDENTIAL_SUBJECT = b"credentialSubject"   # nzcptpl.circom:154-155


def find_cred_subj(bs, pos: int, map_len: int, max_array_len: int, max_map_len: int) -> int:
    """FindCredSubj (nzcptpl.circom:152-226) -> needlePos (not used by NZCPPubIdentity)."""
    found = 0
    p = pos
    for k in range(max_map_len):
        nt, t, v = read_type(bs, p)
        value, np_ = decode_uint(bs, nt, v)
        is_str = int(t == MAJOR_STRING)
        p_next = skip_value(bs, np_ + value * is_str, max_array_len)
        needle = string_equals(bs, np_, value, CREDENTIAL_SUBJECT)
        within = less_than(8, k, map_len)
        found += is_str * needle * within * (np_ + value)
        p = p_next
    return found


def read_cred_subj(bs, pos: int, map_len: int = CREDENTIAL_SUBJECT_MAP_LEN, max_buffer_len: int = NULLIFIER_BYTES):
    """ReadCredSubj (nzcptpl.circom:232-380) -> (given, givenLen, family, familyLen, dob, dobLen)."""
    if map_len != CREDENTIAL_SUBJECT_MAP_LEN:
        raise CircuitError(ERR_RANGE, map_len)
    max_str = max_buffer_len // CREDENTIAL_SUBJECT_MAP_LEN
    flags = []
    copies = []
    p = pos
    for _ in range(CREDENTIAL_SUBJECT_MAP_LEN):
        slen, np_ = read_string_length(bs, p)
        is_g = string_equals(bs, np_, slen, GIVEN_NAME)
        is_f = string_equals(bs, np_, slen, FAMILY_NAME)
        is_d = string_equals(bs, np_, slen, DOB)
        out, p, clen = copy_string(bs, np_ + slen, max_str)
        flags.append((is_g, is_f, is_d))
        copies.append((out, clen))

    def gather(which):
        chars = [sum(flags[i][which] * copies[i][0][h] for i in range(3)) for h in range(max_str)]
        chars += [0] * (max_buffer_len - max_str)
        return chars, sum(flags[i][which] * copies[i][1] for i in range(3))

    g, gl = gather(0)
    f, fl = gather(1)
    d, dl = gather(2)
    return g, gl, f, fl, d, dl


def construct_nullifier(g, gl, f, fl, d, dl, max_buffer_len: int = NULLIFIER_BYTES):
    """ConstructNullifier (nzcptpl.circom:382-433) -> (result, resultLen)."""
    bits = log2(max_buffer_len) + 1
    out = []
    for k in range(max_buffer_len):
        is_g = less_than(bits, k, gl)
        under_sep1 = less_than(bits, k, gl + 1)
        under_fam = less_than(bits, k, gl + 1 + fl)
        under_sep2 = less_than(bits, k, gl + 1 + fl + 1)
        gs = quin_selector(g, k)
        fs = quin_selector(f, k - gl - 1)
        ds = quin_selector(d, k - gl - 1 - fl - 1)
        sep1 = under_sep1 * (1 - is_g)
        fam = under_fam * (1 - under_sep1)
        sep2 = under_sep2 * (1 - under_fam)
        is_d = 1 - under_sep2
        out.append(is_g * gs + sep1 * COMMA + fam * fs + sep2 * COMMA + is_d * ds)
    return out, gl + 1 + fl + 1 + dl


def _field_signed(x: int) -> int:
    x %= R_MOD
    return x - R_MOD if x > R_MOD // 2 else x


class Witness:
    """The semantic signals of one NZCPPubIdentity evaluation (all ints)."""

    def __init__(self):
        self.status = OK
        self.detail = 0
        self.out = [0, 0, 0]
        self.tbs_sha256 = bytes(32)
        self.nullifier_sha512 = bytes(64)
        self.exp = 0
        self.vc_pos = 0
        self.nullifier = bytes(64)
        self.nullifier_len = 0
        self.given_len = self.family_len = self.dob_len = 0


def nzcp_pub_identity(to_be_signed, to_be_signed_len: int, data, is_live: int, max_tbs_bytes: int,
                      max_array_len_vc: int = 0, max_map_len_vc: int = 4) -> Witness:
    """NZCPPubIdentity (nzcptpl.circom:444-655) on field-element inputs.

    to_be_signed: max_tbs_bytes*8 field ints (bits, MSB first per byte);
    to_be_signed_len: field int; data: 160 field ints. Returns a Witness whose
    ``status`` is OK or the first failing check in template order.
    """
    w = Witness()
    try:
        _evaluate(w, to_be_signed, to_be_signed_len, data, is_live, max_tbs_bytes, max_array_len_vc, max_map_len_vc)
    except CircuitError as e:
        w.status, w.detail = e.code, e.detail
    return w


def _evaluate(w, tbs_bits, tbs_len, data, is_live, max_bytes, max_arr, max_map):
    assert max_bytes * 8 <= 4096 and len(tbs_bits) == max_bytes * 8 and len(data) == DATA_BITS
    for i, b in enumerate(tbs_bits):                      # :493-496
        if b % R_MOD not in (0, 1):
            raise CircuitError(ERR_BIT, i)
    ln = _field_signed(tbs_len)                            # :500-505
    if less_than(log2(max_bytes + 1) + 1, ln, max_bytes + 1) != 1:
        raise CircuitError(ERR_LEN, clamp32(ln))
    if ln < 0:
        raise CircuitError(ERR_UNPINNED, clamp32(ln))
    raw = bytes(sum((tbs_bits[k * 8 + 7 - i] % R_MOD) << i for i in range(8)) for k in range(max_bytes))
    w.tbs_sha256 = hashlib.sha256(raw[:ln]).digest()      # :509-517 Sha256Var(3)
    lt_bits = log2(max_bytes) + 1                          # :521-533
    bs = [raw[k] * less_than(lt_bits, k, ln) for k in range(max_bytes)]
    claims_skip = 30 if is_live else 27                    # :474
    map_len, pos = read_map_length(bs, claims_skip)        # :535-538
    vc_pos, exp = find_cwt_claims(bs, pos, map_len, max_arr, max_map)   # :540-546
    w.vc_pos, w.exp = vc_pos, exp
    g, gl, f, fl, d, dl = read_cred_subj(bs, CREDENTIAL_SUBJECT_VC_OFFSET + vc_pos)   # :548-552
    w.given_len, w.family_len, w.dob_len = gl, fl, dl
    res, res_len = construct_nullifier(g, gl, f, fl, d, dl)   # :554-563
    for c in res:                                          # :566-573 Num2Bits(8)
        num2bits_check(8, c)
    w.nullifier = bytes(res)
    w.nullifier_len = res_len
    w.nullifier_sha512 = hashlib.sha512(w.nullifier).digest()   # :577-580 Sha512(512)
    num2bits_check(32, exp)                                # :583-584
    nh, th = w.nullifier_sha512, w.tbs_sha256              # :592-654 packing
    out0 = int.from_bytes(nh[0:31], "big")
    out1 = int.from_bytes(nh[31:32] + th[0:30], "big")
    s2 = int.from_bytes(th[30:32] + exp.to_bytes(4, "big") + bytes(25), "big")
    dsum = sum((x % R_MOD) << j for j, x in enumerate(data))
    out2 = (s2 + (dsum << 40)) % R_MOD
    w.out = [out0, out1, out2]


# ---- input encodings (test/helpers/utils.js:2-89, test/nzcp.js:33-42) --------
def bits_msb_first(bs: bytes):
    return [(b >> (7 - j)) & 1 for b in bs for j in range(8)]


def evm_rearrange(bs: bytes) -> bytes:
    """reversed byte order, reversed bits in each byte (utils.js:73-89)."""
    return bytes(int(f"{b:08b}"[::-1], 2) for b in bs[::-1])


def circuit_input(tbs: bytes, data20: bytes, max_tbs_bytes: int):
    """The reference test's input object: (toBeSigned bits, toBeSignedLen, data bits)."""
    assert len(data20) == 20 and len(tbs) <= max_tbs_bytes
    fitted = tbs + bytes(max_tbs_bytes - len(tbs))
    return bits_msb_first(fitted), len(tbs), bits_msb_first(evm_rearrange(data20))


def expected_public_signals(tbs: bytes, nullifier_str: bytes, exp: int, data20: bytes):
    """The reference test's decode (test/nzcp.js:44-68), run forwards."""
    nh = hashlib.sha512(nullifier_str + bytes(64 - len(nullifier_str))).digest()
    th = hashlib.sha256(tbs).digest()
    return [int.from_bytes(nh[0:31], "big"), int.from_bytes(nh[31:32] + th[0:30], "big"),
            int.from_bytes(th[30:32] + exp.to_bytes(4, "big") + data20 + bytes(5), "big")]
