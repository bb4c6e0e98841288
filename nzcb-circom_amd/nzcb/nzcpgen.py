"""Arithmetization of the reference circuit ``NZCPPubIdentity`` (circuits/nzcp_live.circom:
``NZCPPubIdentity(1, 351, 0, 4, 2, 4)``) with ``nzcb.circuit``: the r1cs that
``snarkjs plonk setup`` turns into ``nzcp_live_final.zkey`` (/root/reference/Makefile:59-62)
and the witness program the GPU runs in place of the circom wasm witness calculator.

Every template follows its circom source statement by statement (file:line on each
function): the same signals, the same ``<==`` / ``===`` constraints and the same
witness rules (circomlib Num2Bits / LessThan / IsZero / IsEqual, QuinSelector,
CalculateTotal). Short linear ``<==`` assignments are substituted, as ``circom --O2``
does (Makefile:12-13).

Two parts come from circuit libraries the reference downloads at build time and which
are not on disk (Makefile:20-43): ``Sha256Var`` (noway/sha256-var-circom)
and ``Sha512`` (Electron-Labs/sha512). They are written here from FIPS 180-4 with
circomlib's gadget shapes (Xor3, Ch, Maj, bit-decomposed modular sums; outputs MSB
first), see ``Circuit.sha_block`` and ``sha256_var``. So the signal order, and with it
the zkey and the proof bytes, are this build's own, not circom's: **parity against
snarkjs on the real nzcp_live.zkey stays unpinned.** What is pinned: the circuit's
public outputs equal the CPU restatement ``oracle/nzcp_circuit.py``, which the
reference's own test vectors pin (test/nzcp.js, test/cbor.js, test/utils.js).
"""
from __future__ import annotations

import functools

from .circuit import (OP_SHA256, OP_SHA512, SHA256_IV, SHA256_SPEC, SHA512_IV, SHA512_SPEC, Circuit, add, lc,
                      scale, sub, w)

# witness failure codes (oracle/nzcp_circuit.py ERR_*, include/nzcb.h NZCB_NZCP_*)
ERR_BIT, ERR_LEN, ERR_RANGE, ERR_SELECT, ERR_NOT_MAP, ERR_UINT23, ERR_NOT_STRING = 1, 2, 3, 4, 5, 6, 7

MAJOR_INT, MAJOR_STRING, MAJOR_ARRAY, MAJOR_MAP = 0, 3, 4, 5

LIVE = dict(is_live=1, max_tbs_bytes=351, max_array_len_vc=0, max_map_len_vc=4)      # nzcp_live.circom:4
EXAMPLE = dict(is_live=0, max_tbs_bytes=314, max_array_len_vc=0, max_map_len_vc=4)   # nzcp_example.circom


def log2(x: int) -> int:
    """log2.circom:5-12 (-1 for 0)."""
    return x.bit_length() - 1


def _template(kind: str):
    """A gadget as a circom component: its signals are named <parent>.<cname>.<signal>
    (cname: the component's name in the caller's template; default <kind>[k]; "" = the
    template is the main itself)."""
    def deco(f):
        @functools.wraps(f)
        def g(c, *args, cname=None, **kw):
            with c.component(kind, cname):
                return f(c, *args, **kw)
        return g
    return deco


class Bytes:
    """A byte array as contiguous wires (``bytes[BytesLen]`` of the cbor templates)."""

    def __init__(self, base: int, n: int):
        self.base, self.n = base, n

    def wires(self) -> list:
        return [w(self.base + k) for k in range(self.n)]


# Names: every template declares its circom signals (Circuit.declare) and passes its
# components' names (cname / name), so the .sym names each signal as circom's does:
# main.<component>[i].<signal>[j] (tests/test_circom_names.py against the reference's
# declarations). Names change no wire, constraint or operation.

# ---------------------------------------------------------------------------- cbortpl
@_template("GetType")
def get_type(c: Circuit, v):
    """GetType (cbortpl.circom:26-52): Num2Bits(8), ShR(8, 5), Bits2Num(3)."""
    c.declare("v", v)
    bits = c.num2bits(v, 8, ERR_RANGE, name="n2b")
    t = c.lin(add(*[scale(bits[5 + i], 1 << i) for i in range(3)]))
    c.declare("type", t)
    c.declare("shr.in", bits)
    c.declare("shr.out", bits[5:])
    c.declare("b2n.in", bits[5:])
    c.declare("b2n.out", t)
    return t


@_template("GetX")
def get_x(c: Circuit, v):
    """GetX (cbortpl.circom:57-72): the 5 low bits of v."""
    c.declare("v", v)
    bits = c.num2bits(v, 8, ERR_RANGE, name="num2Bits")
    x = c.lin(add(*[scale(bits[i], 1 << i) for i in range(5)]))
    c.declare("x", x)
    c.declare("vbits", bits)
    c.declare("b2n.in", bits[:5])
    c.declare("b2n.out", x)
    return x


@_template("GetV")
def get_v(c: Circuit, b: Bytes, pos):
    """GetV (cbortpl.circom:78-90): QuinSelector(BytesLen). Both of QuinSelector's checks
    (the LessThan's Num2Bits and ``lessThan.out === 1``) report ERR_SELECT, as the
    restatement oracle/nzcp_circuit.py quin_selector classifies them."""
    c.declare("pos", pos)
    c.declare("bytes", b.wires())
    v = c.quin(b.n, b.base, b.n, pos, ERR_SELECT, ERR_SELECT, name="quinSelector")
    c.declare("v", v)
    return v


def _tally(c: Circuit, name: str, nums: list, out_name: str | None = None):
    """CalculateTotal(n) (calculate_total.circom, not on disk) over products already
    computed: nums[i], sum = their sum (a signal when longer than two terms)."""
    total = c.lin(add(*nums))
    if out_name:
        c.declare(out_name, total)
    c.declare(f"{name}.nums", nums)
    c.declare(f"{name}.sum", total)
    return total


@_template("DecodeUint23")
def decode_uint23(c: Circuit, v):
    """DecodeUint23 (cbortpl.circom:95-114)."""
    c.declare("v", v)
    x = get_x(c, v, cname="getX")
    lt = c.less_than(x, 24, 8, ERR_RANGE, name="lt")
    c.check_zero(sub(lt, 1), ERR_UINT23)
    c.declare("value", x)
    return x


@_template("DecodeUint")
def decode_uint(c: Circuit, v, b: Bytes, pos):
    """DecodeUint (cbortpl.circom:120-241): every branch is evaluated. Returns (value, nextPos)."""
    c.declare("v", v)
    c.declare("bytes", b.wires())
    c.declare("pos", pos)
    x = get_x(c, v, cname="getX")
    c.declare("x", x)
    cond23 = c.less_than(x, 24, 8, ERR_RANGE, name="lessThan")
    cond24 = c.is_equal(x, 24, name="isEqual24")
    cond25 = c.is_equal(x, 25, name="isEqual25")
    cond26 = c.is_equal(x, 26, name="isEqual26")
    c.declare("condition23", cond23)
    c.declare("condition24", cond24)
    c.declare("condition25", cond25)
    c.declare("condition26", cond26)
    pos = lc(pos)
    value23, next23 = x, pos
    value24 = get_v(c, b, c.mul(cond24, pos), cname="getV_24")
    next24 = add(pos, 1)
    v1_25 = get_v(c, b, c.mul(cond25, pos), cname="getV1_25")
    v2_25 = get_v(c, b, c.mul(cond25, add(pos, 1)), cname="getV2_25")
    value25 = add(scale(v1_25, 256), v2_25)
    next25 = add(pos, 2)
    v26 = [get_v(c, b, c.mul(cond26, add(pos, j)), cname=f"getV{j + 1}_26") for j in range(4)]
    f26 = [1 << 24, 1 << 16, 1 << 8, 1]
    value26 = add(*[scale(v26[j], f26[j]) for j in range(4)])
    next26 = add(pos, 4)
    for sig, val in (("value23", value23), ("nextPos23", next23), ("value24", value24), ("nextPos24", next24),
                     ("value1_25", scale(v1_25, 256)), ("value2_25", v2_25), ("value25", value25),
                     ("nextPos25", next25), ("value1_26", scale(v26[0], f26[0])),
                     ("value2_26", scale(v26[1], f26[1])), ("value3_26", scale(v26[2], f26[2])),
                     ("value4_26", v26[3]), ("value26", value26), ("nextPos26", next26)):
        c.declare(sig, val)
    nums = [c.mul(cond23, value23), c.mul(cond24, value24), c.mul(cond25, value25), c.mul(cond26, value26)]
    value = _tally(c, "valueTally", nums, "value")
    nums = [c.mul(cond23, next23), c.mul(cond24, next24), c.mul(cond25, next25), c.mul(cond26, next26)]
    next_pos = _tally(c, "nextPosTally", nums, "nextPos")
    return value, next_pos


@_template("ReadType")
def read_type(c: Circuit, b: Bytes, pos):
    """ReadType (cbortpl.circom:246-261). Returns (nextPos, type, v)."""
    c.declare("bytes", b.wires())
    c.declare("pos", pos)
    v = get_v(c, b, pos, cname="getV")
    c.declare("v", v)
    typ = get_type(c, v, cname="getType")
    c.declare("type", typ)
    c.declare("nextPos", add(pos, 1))
    return add(pos, 1), typ, v


@_template("SkipValueScalar")
def skip_value_scalar(c: Circuit, b: Bytes, pos):
    """SkipValueScalar (cbortpl.circom:266-297): ints and strings."""
    c.declare("bytes", b.wires())
    c.declare("pos", pos)
    nxt, typ, v = read_type(c, b, pos, cname="readType")
    value, dnext = decode_uint(c, v, b, nxt, cname="decodeUint")
    is_int = c.is_equal(typ, MAJOR_INT, name="isInt")
    is_string = c.is_equal(typ, MAJOR_STRING, name="isString")
    nums = [c.mul(is_int, dnext), c.mul(is_string, add(dnext, value))]
    return _tally(c, "calculateTotal", nums, "nextPos")


@_template("SkipValue")
def skip_value(c: Circuit, b: Bytes, pos, max_array_len: int):
    """SkipValue (cbortpl.circom:306-366): SkipValueScalar's ints and strings plus arrays of
    up to MaxArrayLen scalars. Every element slot i runs a SkipValueScalar from the previous
    slot's end, gated by shouldConsider[i] = isArray * (i < isArray * len); a
    QuinSelector(MaxArrayLen) picks the end of element len - 1. nzcp_live has
    MaxArrayLen = 0: no loop, and QuinSelector(0) outputs 0 (quinSelector.circom:19-41)."""
    c.declare("bytes", b.wires())
    c.declare("pos", pos)
    nxt, typ, v = read_type(c, b, pos, cname="readType")
    value, dnext = decode_uint(c, v, b, nxt, cname="decodeUint")
    is_int = c.is_equal(typ, MAJOR_INT, name="isInt")
    is_string = c.is_equal(typ, MAJOR_STRING, name="isString")
    is_array = c.is_equal(typ, MAJOR_ARRAY, name="isArray")
    arr_len = c.mul(is_array, value) if max_array_len else None     # lt[i].in[1] <== isArray.out * value
    ends = c.alloc(max_array_len)                                   # nextPosArray[i] = qs.in[i]
    c.declare("nextPosArray", [w(ends + i) for i in range(max_array_len)])
    prev = dnext
    bits = log2(max_array_len) + 1
    for i in range(max_array_len):
        lt = c.less_than(i, arr_len, bits, ERR_RANGE, name=f"lt[{i}]")
        consider = c.mul(is_array, lt)                              # shouldConsider[i]
        c.declare(f"shouldConsider[{i}]", consider)
        end = skip_value_scalar(c, b, c.mul(prev, consider), cname=f"skipValue[{i}]")
        c.lin(end, dst=ends + i)
        prev = w(ends + i)
    index = c.mul(is_array, sub(value, 1))     # qs.index <== isArray.out * (decodeUint.value - 1)
    nums = [c.mul(is_int, dnext), c.mul(is_string, add(dnext, value))]
    if max_array_len:
        nums.append(c.mul(is_array, c.quin(max_array_len, ends, max_array_len, index, ERR_SELECT, ERR_SELECT,
                                           name="qs")))
    else:       # QuinSelector(0): no inputs, out = 0 (its LessThan is declared, not wired)
        c.declare("qs.index", index)
        c.declare("qs.out", 0)
        c.declare("qs.lessThan.in", [0, 0])
        nums.append(0)
    return _tally(c, "calculateTotal", nums, "nextPos")


@_template("StringEquals")
def string_equals(c: Circuit, b: Bytes, const: list, pos, length):
    """StringEquals (cbortpl.circom:373-404)."""
    c.declare("bytes", b.wires())
    c.declare("pos", pos)
    c.declare("len", length)
    is_same_len = c.is_equal(length, len(const), name="isSameLen")
    cond = [is_same_len]
    for i, ch in enumerate(const):
        cond.append(c.is_equal(ch, get_v(c, b, add(pos, i), cname=f"getV[{i}]"), name=f"isEqual[{i}]"))
    out = c.is_zero(sub(len(const) + 1, add(*cond)), name="isZero")
    c.declare("out", out)
    return out


@_template("ReadStringLength")
def read_string_length(c: Circuit, b: Bytes, pos):
    """ReadStringLength (cbortpl.circom:410-428). Returns (len, nextPos = pos + 1)."""
    c.declare("bytes", b.wires())
    c.declare("pos", pos)
    nxt, typ, v = read_type(c, b, pos, cname="readType")
    c.check_zero(sub(typ, MAJOR_STRING), ERR_NOT_STRING)
    value, _ = decode_uint(c, v, b, nxt, cname="dUint")
    c.declare("len", value)
    c.declare("nextPos", nxt)
    return value, nxt


@_template("ReadMapLength")
def read_map_length(c: Circuit, b: Bytes, pos):
    """ReadMapLength (cbortpl.circom:434-453). Returns (len, nextPos)."""
    c.declare("pos", pos)
    c.declare("bytes", b.wires())
    nxt, typ, v = read_type(c, b, pos, cname="readType")
    c.check_zero(sub(typ, MAJOR_MAP), ERR_NOT_MAP)
    length = decode_uint23(c, v, cname="dUint23")
    c.declare("len", length)
    c.declare("nextPos", nxt)
    return length, nxt


@_template("CopyString")
def copy_string(c: Circuit, b: Bytes, pos, max_len: int, out_base: int | None = None):
    """CopyString (cbortpl.circom:460-503). Returns (outbytes, nextPos, len)."""
    c.declare("bytes", b.wires())
    c.declare("pos", pos)
    length, nxt = read_string_length(c, b, pos, cname="readStrLen")
    bits = log2(max_len) + 1
    out = []
    for i in range(max_len):
        v = get_v(c, b, add(nxt, i), cname=f"getV[{i}]")
        lt = c.less_than(i, length, bits, ERR_RANGE, name=f"lt[{i}]")
        out.append(c.mul(v, lt))
    c.declare("outbytes", out)
    c.declare("nextPos", add(nxt, length))
    c.declare("len", length)
    return out, add(nxt, length), length


# --------------------------------------------------------------------------- nzcptpl
@_template("FindCWTClaims")
def find_cwt_claims(c: Circuit, b: Bytes, map_len, pos, max_array_len: int, max_map_len: int):
    """FindCWTClaims (nzcptpl.circom:33-145). Returns (vcPos, exp)."""
    vc = [118, 99]
    c.declare("mapLen", map_len)
    c.declare("bytes", b.wires())
    c.declare("pos", pos)
    found, exp_pos = [], []
    for k in range(max_map_len):
        nxt, typ, v = read_type(c, b, pos, cname=f"readType[{k}]")
        c.declare(f"v[{k}]", v)
        c.declare(f"type[{k}]", typ)
        value, dnext = decode_uint(c, v, b, nxt, cname=f"decodeUint[{k}]")
        c.declare(f"value[{k}]", value)
        is_string = c.is_equal(typ, MAJOR_STRING, name=f"isString[{k}]")
        is_int = c.is_equal(typ, MAJOR_INT, name=f"isInt[{k}]")
        skip_pos = c.mul(value, is_string, dnext)
        next_pos = skip_value(c, b, skip_pos, max_array_len, cname=f"skipValue[{k}]")   # runs once its inputs are set
        needle = string_equals(c, b, vc, dnext, value, cname=f"isNeedleString[{k}]")
        is4 = c.is_equal(4, value, name=f"is4Int[{k}]")
        within = c.less_than(k, map_len, 8, ERR_RANGE, name=f"withinMapLen[{k}]")
        is_needle = c.mul(is_string, needle)
        is_exp = c.mul(is_int, is4)
        accepted = c.mul(is_needle, within)
        exp_accepted = c.mul(is_exp, within)
        for sig, val in (("isNeedle", is_needle), ("isExp", is_exp), ("isAccepted", accepted),
                         ("isExpAccepted", exp_accepted)):
            c.declare(f"{sig}[{k}]", val)
        found.append(c.mul(accepted, add(dnext, value)))
        exp_pos.append(c.mul(exp_accepted, dnext))
        pos = next_pos
    vc_pos = _tally(c, "foundPosTally", found, "vcPos")
    epos = _tally(c, "expPosTally", exp_pos)
    nxt, _, v = read_type(c, b, epos, cname="expReadType")
    exp, _ = decode_uint(c, v, b, nxt, cname="expDecodeUint")
    c.declare("exp", exp)
    return vc_pos, exp


@_template("FindCredSubj")
def find_cred_subj(c: Circuit, b: Bytes, map_len, pos, max_array_len: int, max_map_len: int):
    """FindCredSubj (nzcptpl.circom:152-226; not used by NZCPPubIdentity, tested by the
    reference at test/nzcp.js:144-215). Returns needlePos, the position of the
    "credentialSubject" key's value."""
    needle_str = [99, 114, 101, 100, 101, 110, 116, 105, 97, 108, 83, 117, 98, 106, 101, 99, 116]
    c.declare("mapLen", map_len)
    c.declare("bytes", b.wires())
    c.declare("pos", pos)
    found = []
    for k in range(max_map_len):
        nxt, typ, v = read_type(c, b, pos, cname=f"readType[{k}]")
        c.declare(f"v[{k}]", v)
        c.declare(f"type[{k}]", typ)
        value, dnext = decode_uint(c, v, b, nxt, cname=f"decodeUint[{k}]")
        c.declare(f"value[{k}]", value)
        is_string = c.is_equal(typ, MAJOR_STRING, name=f"isString[{k}]")
        next_pos = skip_value(c, b, c.mul(value, is_string, dnext), max_array_len, cname=f"skipValue[{k}]")
        needle = string_equals(c, b, needle_str, dnext, value, cname=f"isNeedleString[{k}]")
        within = c.less_than(k, map_len, 8, ERR_RANGE, name=f"withinMapLen[{k}]")
        is_needle = c.mul(is_string, needle)
        accepted = c.mul(is_needle, within)
        c.declare(f"isNeedle[{k}]", is_needle)
        c.declare(f"isAccepted[{k}]", accepted)
        found.append(c.mul(accepted, add(dnext, value)))
        pos = next_pos
    return _tally(c, "foundPosTally", found, "needlePos")


@_template("ReadCredSubj")
def read_cred_subj(c: Circuit, b: Bytes, pos, max_buffer_len: int, map_len=None):
    """ReadCredSubj (nzcptpl.circom:232-360). Returns ((givenName base, len), (familyName ...),
    (dob ...)); each name is max_buffer_len / 3 contiguous signals (zeros past them).
    map_len: the mapLen input, checked against 3 (``hardcore_assert``, :261); NZCPPubIdentity
    passes the constant 3 (:552), which leaves no constraint."""
    n_map = 3
    c.declare("mapLen", n_map if map_len is None else map_len)
    c.declare("bytes", b.wires())
    c.declare("pos", pos)
    if map_len is not None:
        c.check_zero(sub(map_len, n_map), ERR_RANGE)
    max_str = max_buffer_len // n_map
    given = [103, 105, 118, 101, 110, 78, 97, 109, 101]
    family = [102, 97, 109, 105, 108, 121, 78, 97, 109, 101]
    dob = [100, 111, 98]
    is_g, is_f, is_d, copies = [], [], [], []
    for k in range(n_map):
        length, nxt = read_string_length(c, b, pos, cname=f"readStringLength[{k}]")
        is_g.append(string_equals(c, b, given, nxt, length, cname=f"isGivenName[{k}]"))
        is_f.append(string_equals(c, b, family, nxt, length, cname=f"isFamilyName[{k}]"))
        is_d.append(string_equals(c, b, dob, nxt, length, cname=f"isDOB[{k}]"))
        out, pos, ln = copy_string(c, b, add(nxt, length), max_str, cname=f"copyString[{k}]")
        copies.append((out, ln))
    res = []
    for sel, nm in ((is_g, "givenName"), (is_f, "familyName"), (is_d, "dob")):
        base = c.alloc(max_str)
        prods = [[c.mul(sel[i], copies[i][0][h]) for i in range(n_map)] for h in range(max_str)]
        for h in range(max_str):
            c.lin(add(*prods[h]), dst=base + h)
        c.declare(nm, [w(base + h) for h in range(max_str)] + [0] * (max_buffer_len - max_str))
        for h in range(max_str):
            c.declare(f"{nm}CharTally[{h}].nums", prods[h])
            c.declare(f"{nm}CharTally[{h}].sum", w(base + h))
        ln = _tally(c, f"{nm}LenTally", [c.mul(sel[i], copies[i][1]) for i in range(n_map)], f"{nm}Len")
        res.append((base, ln))
    return res, max_str


@_template("ConstructNullifier")
def construct_nullifier(c: Circuit, names, max_str: int, max_buffer_len: int):
    """ConstructNullifier (nzcptpl.circom:364-440). Returns the result[] LCs."""
    comma = 44
    bits = log2(max_buffer_len) + 1
    (gb, gl), (fb, fl), (db, dl) = names
    for nm, base, ln in (("givenName", gb, gl), ("familyName", fb, fl), ("dob", db, dl)):
        c.declare(nm, [w(base + h) if h < max_str else 0 for h in range(max_buffer_len)])
        c.declare(f"{nm}Len", ln)
    result = []
    for k in range(max_buffer_len):
        is_given = c.less_than(k, gl, bits, ERR_RANGE, name=f"isGivenName[{k}]")
        under_sep1 = c.less_than(k, add(gl, 1), bits, ERR_RANGE, name=f"isUnderSep1[{k}]")
        under_family = c.less_than(k, add(gl, 1, fl), bits, ERR_RANGE, name=f"isUnderFamilyName[{k}]")
        under_sep2 = c.less_than(k, add(gl, 1, fl, 1), bits, ERR_RANGE, name=f"isUnderSep2[{k}]")
        g_sel = c.quin(max_buffer_len, gb, max_str, k, ERR_SELECT, ERR_SELECT, name=f"givenNameSelector[{k}]")
        f_sel = c.quin(max_buffer_len, fb, max_str, sub(sub(k, gl), 1), ERR_SELECT, ERR_SELECT,
                       name=f"familyNameSelector[{k}]")
        d_sel = c.quin(max_buffer_len, db, max_str, sub(sub(sub(sub(k, gl), 1), fl), 1), ERR_SELECT, ERR_SELECT,
                       name=f"dobSelector[{k}]")
        not_given = sub(1, is_given)
        is_sep1 = c.mul(under_sep1, not_given)
        is_family = c.mul(under_family, sub(1, under_sep1))
        is_sep2 = c.mul(under_sep2, sub(1, under_family))
        is_dob = sub(1, under_sep2)
        given_char = c.mul(is_given, g_sel)
        family_char = c.mul(is_family, f_sel)
        dob_char = c.mul(is_dob, d_sel)
        result.append(c.lin(add(given_char, scale(is_sep1, comma), family_char, scale(is_sep2, comma), dob_char),
                            force=True))
        for sig, val in (("notGivenName", not_given), ("isSep1", is_sep1), ("isFamilyName", is_family),
                         ("isSep2", is_sep2), ("isDOB", is_dob), ("givenNameChar", given_char),
                         ("sep1Char", scale(is_sep1, comma)), ("familyNameChar", family_char),
                         ("sep2Char", scale(is_sep2, comma)), ("dobChar", dob_char), ("result", result[-1])):
            c.declare(f"{sig}[{k}]", val)
    c.declare("resultLen", add(gl, 1, fl, 1, dl))
    return result


def msg_word_bits(base: int, t: int, bits: int) -> list:
    """Bit-LCs (LSB first) of message word t over byte wires with LSB-first bits
    (wire of byte k, bit j = base + 8k + j); words are big-endian, as in FIPS 180-4."""
    nb = bits // 8
    out = []
    for i in range(bits):
        m = bits - 1 - i                 # MSB-first index inside the word
        byte = nb * t + m // 8
        out.append(w(base + 8 * byte + 7 - m % 8))
    return out


@_template("Sha256Var")
def sha256_var(c: Circuit, msg_bits_msb: list, len_bytes, block_space: int):
    """Sha256Var(BlockSpace) (noway/sha256-var-circom, not on disk; used at
    nzcptpl.circom:509-517): SHA-256 of the first ``len_bytes`` bytes of the input bits,
    with the input beyond the length masked out. Written from FIPS 180-4:

    * isLen[k] = IsEqual(k, len) for every byte position; lt[k] = (k < len) as a running
      sum; Num2Bits(9) of len for the 64-bit length field (len < 512 bytes);
    * padded byte-wise bits p (LSB first within a byte): message bit * lt[k], the 0x80
      byte at k = len, and the length field in bytes 62..63 of the last block, selected
      by isLast[b] = sum of isLen over [64b - 8, 64b + 56);
    * all 2^BlockSpace compressions chained; the digest is sum_b isLast[b] * H_b
      (a running sum, as QuinSelector's). Output bits MSB first (circomlib's order)."""
    nblocks = 1 << block_space
    nbytes = 64 * nblocks
    L = lc(len_bytes)
    lbits = c.num2bits(L, 9, ERR_RANGE)
    is_len = [c.is_equal(k, L) for k in range(nbytes)]
    lt_base = c.alloc(nbytes)
    prev = 1
    for k in range(nbytes):
        c.lin(sub(prev, is_len[k]), dst=lt_base + k)
        prev = w(lt_base + k)
    last = []
    for b in range(nblocks):
        terms = [is_len[k] for k in range(max(0, 64 * b - 8), min(nbytes, 64 * b + 56))]
        last.append(c.lin(add(*terms), force=True))
    lf = [[c.mul(last[b], lbits[i]) for i in range(9)] for b in range(nblocks)]
    pbase = c.alloc(8 * nbytes)
    for k in range(nbytes):
        b, off = divmod(k, 64)
        for j in range(8):
            extra = {}
            if j == 7:
                extra = add(extra, is_len[k])
            if off == 63 and j >= 3:
                extra = add(extra, lf[b][j - 3])
            if off == 62 and j <= 3:
                extra = add(extra, lf[b][5 + j])
            src = 8 * k + 7 - j
            bit = msg_bits_msb[src] if src < len(msg_bits_msb) else 0
            c.mul(bit, w(lt_base + k), extra, dst=pbase + 8 * k + j)
    state, prev_base, hs = list(SHA256_IV), None, []
    for b in range(nblocks):
        mb = pbase + 512 * b
        words = [msg_word_bits(mb, t, 32) for t in range(16)]
        base, state = c.sha_block(SHA256_SPEC, state, words, OP_SHA256, (prev_base, mb))
        prev_base = base
        hs.append(state)
    out = []
    for j in range(8):
        for k in range(32):
            i = 31 - k
            acc = 0
            for b in range(nblocks):
                acc = c.mul(last[b], hs[b][j][i], acc)
            out.append(acc)
    return out


@_template("Sha512")
def sha512_64(c: Circuit, byte_base: int):
    """Sha512(512) (Electron-Labs/sha512, not on disk; used at nzcptpl.circom:577-580) for
    a 64-byte message over byte wires with LSB-first bits: one block, constant padding
    (0x80, zeros, 128-bit length 512). Output bits MSB first."""
    words = [msg_word_bits(byte_base, t, 64) for t in range(8)]
    words += [1 << 63] + [0] * 6 + [512]
    _, H = c.sha_block(SHA512_SPEC, list(SHA512_IV), words, OP_SHA512, (None, byte_base))
    return [H[j][63 - k] for j in range(8) for k in range(64)]


def nzcp_pub_identity(is_live: int, max_tbs_bytes: int, max_array_len_vc: int, max_map_len_vc: int,
                      max_array_len_cs: int = 2, max_map_len_cs: int = 4) -> Circuit:
    """NZCPPubIdentity (nzcptpl.circom:444-655). Wires: 1, out[3], toBeSigned[8 * Max],
    toBeSignedLen, data[160] (circom's order: outputs, then inputs as declared)."""
    chunk_bits, byte_bits, data_len = 248, 8, 160
    chunk_bytes = chunk_bits // byte_bits
    claims_skip = 30 if is_live else 27
    cred_subj_offset, null_bytes = 171, 64
    max_bits = 8 * max_tbs_bytes
    c = Circuit(3, 0, max_bits + 1 + data_len,
                input_names=[("toBeSigned", max_bits), ("toBeSignedLen", 1), ("data", data_len)])
    tbs = [w(c.in_base + i) for i in range(max_bits)]
    tbs_len = w(c.in_base + max_bits)
    data = [w(c.in_base + max_bits + 1 + i) for i in range(data_len)]
    # bit checks (:493-496)
    for i in range(max_bits):
        c.check_quad(tbs[i], sub(tbs[i], 1), ERR_BIT)
    # toBeSignedLen < Max + 1 (:500-505)
    lt_max = c.less_than(tbs_len, max_tbs_bytes + 1, log2(max_tbs_bytes + 1) + 1, ERR_RANGE,
                         name="lteMaxToBeSignedBytes")
    c.check_zero(sub(lt_max, 1), ERR_LEN)
    # SHA-256 of ToBeSigned (:509-517)
    sha256 = sha256_var(c, tbs, tbs_len, 3, cname="tbsSha256")
    # bits -> bytes, zero past the length (:521-533)
    tb = c.alloc(max_tbs_bytes, "ToBeSigned")
    bits = log2(max_tbs_bytes) + 1
    for k in range(max_tbs_bytes):
        b2n = add(*[scale(tbs[8 * k + 7 - i], 1 << i) for i in range(8)])
        c.declare(f"b2n[{k}].in", [tbs[8 * k + 7 - i] for i in range(8)])
        c.declare(f"b2n[{k}].out", b2n)
        lt = c.less_than(k, tbs_len, bits, ERR_RANGE, name=f"ltLen[{k}]")
        c.mul(b2n, lt, dst=tb + k)
    tbytes = Bytes(tb, max_tbs_bytes)
    map_len, nxt = read_map_length(c, tbytes, claims_skip, cname="readMapLengthClaims")
    vc_pos, exp = find_cwt_claims(c, tbytes, map_len, nxt, max_array_len_vc, max_map_len_vc, cname="findVC")
    names, max_str = read_cred_subj(c, tbytes, add(vc_pos, cred_subj_offset), null_bytes, cname="readCredSubj")
    result = construct_nullifier(c, names, max_str, null_bytes, cname="nullifier")
    nb = [c.num2bits(result[k], 8, ERR_RANGE, name=f"n2bNullifier[{k}]") for k in range(null_bytes)]
    nbase = next(iter(nb[0][0]))            # byte wires: nbase + 8k + j (LSB-first bits)
    sha512 = sha512_64(c, nbase, cname="nullifierSha512")
    c.declare("exp", exp)
    c.declare("nullifierBits", sha512)
    exp_bits = c.num2bits(exp, 32, ERR_RANGE, name="n2bExp")
    ins = [[0] * chunk_bits for _ in range(3)]
    for k in range(chunk_bytes):                                   # nullifier hash part (:596-601)
        b = chunk_bytes - 1 - k
        for i in range(byte_bits):
            ins[0][b * byte_bits + (7 - i)] = sha512[k * byte_bits + i]
    for k in range(8 // byte_bits):                                # (:602-607)
        b = chunk_bytes - 1 - k
        for i in range(byte_bits):
            ins[1][b * byte_bits + (7 - i)] = sha512[chunk_bits + k * byte_bits + i]
    for k in range(1, chunk_bytes):                                # ToBeSigned sha256 (:610-615)
        b = chunk_bytes - 1 - k
        for i in range(byte_bits):
            ins[1][b * byte_bits + (7 - i)] = sha256[(k * byte_bits + i) - 8]
    for k in range(16 // byte_bits):                               # (:616-621)
        b = chunk_bytes - 1 - k
        for i in range(byte_bits):
            ins[2][b * byte_bits + (7 - i)] = sha256[chunk_bits + (k * byte_bits + i) - 8]
    for idx, k in enumerate(range(2, 2 + 4)):                      # exp (:626-634)
        b = chunk_bytes - 1 - k
        d = 4 - 1 - idx
        for i in range(byte_bits):
            ins[2][b * byte_bits + i] = exp_bits[d * byte_bits + i]
    for idx, k in enumerate(range(2 + 4, chunk_bytes)):            # pass-through data (:637-651)
        b = chunk_bytes - 1 - k
        for i in range(byte_bits):
            if idx < data_len // byte_bits:
                d = data_len // byte_bits - 1 - idx
                ins[2][b * byte_bits + i] = data[d * byte_bits + i]
    for j in range(3):                                             # Bits2Num(248) -> out (:653-655)
        c.lin(add(*[scale(x, 1 << i) if isinstance(x, dict) else 0 for i, x in enumerate(ins[j])]),
              dst=c.out_wires[j])
        c.declare(f"outB2n[{j}].in", [x if isinstance(x, dict) else 0 for x in ins[j]])
        c.declare(f"outB2n[{j}].out", w(c.out_wires[j]))
    return c


# ------------------------------------------------------------ the reference's test mains
# The wrapper circuits the reference's tests compile (/root/reference/circuits/*_test.circom,
# *Test.circom), built from the same gadgets as NZCPPubIdentity: main's outputs first, then
# its inputs in declaration order (circom's wire order), so witness[1..] is what the
# reference's tests read (test/cbor.js, test/quinSelector.js, test/nzcp.js).
WRAPPERS = {
    "getType_test": ("GetType", ()),
    "getX_test": ("GetX", ()),
    "getV3_test": ("GetV", (3,)),
    "getV4_test": ("GetV", (4,)),
    "getV5_test": ("GetV", (5,)),
    "decodeUint32_test": ("DecodeUint23", ()),
    "decodeUint_test": ("DecodeUint", (4,)),
    "readType_test": ("ReadType", (3,)),
    "skipValueScalar_test": ("SkipValueScalar", (5,)),
    "skipValue5_test": ("SkipValue", (5, 4)),
    "skipValue6_test": ("SkipValue", (6, 4)),
    "stringEquals_test": ("StringEquals", (5, (97, 98, 99, 100, 101), 5)),
    "readStringLength_test": ("ReadStringLength", (5,)),
    "readMapLength_test": ("ReadMapLength", (7,)),
    "copyString_test": ("CopyString", (5, 4)),
    "quinSelector0_test": ("QuinSelector", (0,)),
    "quinSelector1_test": ("QuinSelector", (1,)),
    "quinSelector2_test": ("QuinSelector", (2,)),
    "quinSelector3_test": ("QuinSelector", (3,)),
    "quinSelector4_test": ("QuinSelector", (4,)),
    "quinSelector5_test": ("QuinSelector", (5,)),
    "findCWTClaims_exampleTest": ("FindCWTClaims", (314, 0, 4)),
    "findCWTClaims_liveTest": ("FindCWTClaims", (351, 0, 4)),
    "findCredSubj_exampleTest": ("FindCredSubj", (314, 2, 4)),
    "findCredSubj_liveTest": ("FindCredSubj", (351, 2, 4)),
    "readCredSubj_exampleTest": ("ReadCredSubj", (314, 32)),
    "readCredSubj_liveTest": ("ReadCredSubj", (351, 64)),
    "constructNullifier_test": ("ConstructNullifier", (64,)),
}


def template_circuit(template: str, *params) -> Circuit:
    """``component main = <template>(<params>)`` as an r1cs + witness program. Inputs are
    private (circom's default for main), named as the template declares them."""
    def io(outs, ins):
        n_out = sum(k for _, k in outs)
        c = Circuit(n_out, 0, sum(k for _, k in ins), input_names=list(ins), output_names=list(outs))
        wires, o = {}, c.in_base
        for name, k in ins:
            wires[name] = o
            o += k
        return c, wires

    def put(c, values):
        """main's outputs (LCs or ints), in declaration order"""
        for i, x in enumerate(values):
            c.lin(lc(x), dst=c.out_wires[i])

    if template in ("GetType", "GetX", "DecodeUint23"):
        c, wi = io([({"GetType": "type", "GetX": "x"}.get(template, "value"), 1)], [("v", 1)])
        fn = {"GetType": get_type, "GetX": get_x, "DecodeUint23": decode_uint23}[template]
        put(c, [fn(c, w(wi["v"]), cname="")])
    elif template == "GetV":
        (n,) = params
        c, wi = io([("v", 1)], [("bytes", n), ("pos", 1)])
        put(c, [get_v(c, Bytes(wi["bytes"], n), w(wi["pos"]), cname="")])
    elif template == "DecodeUint":
        (n,) = params
        c, wi = io([("value", 1), ("nextPos", 1)], [("v", 1), ("bytes", n), ("pos", 1)])
        put(c, list(decode_uint(c, w(wi["v"]), Bytes(wi["bytes"], n), w(wi["pos"]), cname="")))
    elif template == "ReadType":
        (n,) = params
        c, wi = io([("nextPos", 1), ("type", 1), ("v", 1)], [("bytes", n), ("pos", 1)])
        put(c, list(read_type(c, Bytes(wi["bytes"], n), w(wi["pos"]), cname="")))
    elif template in ("SkipValueScalar", "SkipValue"):
        n = params[0]
        c, wi = io([("nextPos", 1)], [("bytes", n), ("pos", 1)])
        b, pos = Bytes(wi["bytes"], n), w(wi["pos"])
        put(c, [skip_value_scalar(c, b, pos, cname="") if template == "SkipValueScalar"
                else skip_value(c, b, pos, params[1], cname="")])
    elif template == "StringEquals":
        n, const, clen = params
        c, wi = io([("out", 1)], [("bytes", n), ("pos", 1), ("len", 1)])
        put(c, [string_equals(c, Bytes(wi["bytes"], n), list(const[:clen]), w(wi["pos"]), w(wi["len"]), cname="")])
    elif template == "ReadStringLength":
        (n,) = params
        c, wi = io([("len", 1), ("nextPos", 1)], [("bytes", n), ("pos", 1)])
        put(c, list(read_string_length(c, Bytes(wi["bytes"], n), w(wi["pos"]), cname="")))
    elif template == "ReadMapLength":
        (n,) = params
        c, wi = io([("len", 1), ("nextPos", 1)], [("pos", 1), ("bytes", n)])
        put(c, list(read_map_length(c, Bytes(wi["bytes"], n), w(wi["pos"]), cname="")))
    elif template == "CopyString":
        n, max_len = params
        c, wi = io([("outbytes", max_len), ("nextPos", 1), ("len", 1)], [("bytes", n), ("pos", 1)])
        out, nxt, ln = copy_string(c, Bytes(wi["bytes"], n), w(wi["pos"]), max_len, cname="")
        put(c, out + [nxt, ln])
    elif template == "QuinSelector":
        (n,) = params
        c, wi = io([("out", 1)], [("in", n), ("index", 1)])
        if n:
            put(c, [c._quin(n, wi["in"], n, w(wi["index"]), ERR_SELECT, ERR_SELECT)])
        else:   # QuinSelector(0): no range check, out <== 0 (quinSelector.circom:21, 41)
            put(c, [0])
    elif template in ("FindCWTClaims", "FindCredSubj"):
        n, max_arr, max_map = params
        outs = [("vcPos", 1), ("exp", 1)] if template == "FindCWTClaims" else [("needlePos", 1)]
        c, wi = io(outs, [("mapLen", 1), ("bytes", n), ("pos", 1)])
        args = (c, Bytes(wi["bytes"], n), w(wi["mapLen"]), w(wi["pos"]), max_arr, max_map)
        put(c, list(find_cwt_claims(*args, cname="")) if template == "FindCWTClaims"
            else [find_cred_subj(*args, cname="")])
    elif template == "ReadCredSubj":
        n, max_buf = params
        outs = [("givenName", max_buf), ("givenNameLen", 1), ("familyName", max_buf), ("familyNameLen", 1),
                ("dob", max_buf), ("dobLen", 1)]
        c, wi = io(outs, [("mapLen", 1), ("bytes", n), ("pos", 1)])
        names, max_str = read_cred_subj(c, Bytes(wi["bytes"], n), w(wi["pos"]), max_buf, map_len=w(wi["mapLen"]),
                                        cname="")
        vals = []
        for base, ln in names:
            vals += [w(base + h) for h in range(max_str)] + [0] * (max_buf - max_str) + [ln]
        put(c, vals)
    elif template == "ConstructNullifier":
        (max_buf,) = params
        ins = [("givenName", max_buf), ("givenNameLen", 1), ("familyName", max_buf), ("familyNameLen", 1),
               ("dob", max_buf), ("dobLen", 1)]
        c, wi = io([("result", max_buf), ("resultLen", 1)], ins)
        names = [(wi[k], w(wi[k + "Len"])) for k in ("givenName", "familyName", "dob")]
        result = construct_nullifier(c, names, max_buf, max_buf, cname="")
        total = add(*[ln for _, ln in names], 2)       # resultLen (nzcptpl.circom:432)
        put(c, result + [total])
    else:
        raise ValueError(f"unknown template {template}")
    return c


def wrapper_circuit(name: str) -> Circuit:
    """One of the reference's test mains by file stem (WRAPPERS), e.g. "skipValue5_test"."""
    template, params = WRAPPERS[name]
    return template_circuit(template, *params)
