"""The reference's gadget known-answer tests run through the r1cs generator (VERDICT r2
item 4): every wrapper main of /root/reference/circuits/*_test.circom and *Test.circom is
built from nzcb/nzcpgen.py's gadgets (nzcpgen.wrapper_circuit), its witness program is
evaluated on the CPU (oracle/wvm.py), and

* every positive KAT of test/cbor.js, test/quinSelector.js and test/nzcp.js:98-368 gives
  the reference's expected outputs at witness[1..] AND satisfies every r1cs constraint;
* every negative KAT (test/cbor.js:123 DecodeUint23 of x > 23, test/quinSelector.js:63-87
  index = choices) is rejected by the witness program, AND the witness carried past the
  failure violates the r1cs: the rejection is a constraint, not only a calculator check;
* soundness probe: on the accepted witnesses, changing any single signal (except an IsZero
  inverse of a zero input, which circomlib leaves free) violates some constraint, and
  tampered selectors (a QuinSelector pointing at another element, an IsZero output
  flipped) are rejected.

The expected values are the reference's literal KATs; where a test needs a pass the
reference reads from env secrets (LIVE_PASS_URI_1..4) a live-shaped pass stands in and
the KAT positions (vcPos 80, credential subject 250, test/nzcp.js:117,164,207) still hold.
"""
import random

import pytest

import nzcp_cases as C
from nzcb import circuit, nzcp, nzcpgen
from oracle import nzcp_circuit as nz
from oracle import wvm

R = circuit.R
_CACHE = {}


def built(name):
    if name not in _CACHE:
        c = nzcpgen.wrapper_circuit(name)
        _CACHE[name] = (c, c.write_program(), _wire_index(c))
    return _CACHE[name]


def _wire_index(c):
    idx = {}
    for k, cons in enumerate(c.constraints):
        for part in cons:
            for wire in part:
                if wire:
                    idx.setdefault(wire, set()).add(k)
    return idx


def _violated(c, wit, ks):
    bad = []
    for k in ks:
        A, B, Cc = c.constraints[k]
        a = sum(v * wit[i] for i, v in A.items()) % R
        b = sum(v * wit[i] for i, v in B.items()) % R
        cc = sum(v * wit[i] for i, v in Cc.items()) % R
        if (a * b - cc) % R:
            bad.append(k)
    return bad


def unsat(c, wit):
    return _violated(c, wit, range(len(c.constraints)))


def run(name, inputs):
    c, prog, _ = built(name)
    wit, fail = wvm.evaluate(prog, [x % R for x in inputs])
    return c, wit, fail


def accept(name, inputs):
    """Positive KAT: no failure, every constraint holds; returns the outputs."""
    c, wit, fail = run(name, inputs)
    assert fail is None, (name, fail)
    assert unsat(c, wit) == [], name
    return wit[1:1 + c.n_out]


def reject(name, inputs):
    """Negative KAT: the calculator rejects AND the carried-past witness violates the r1cs."""
    c, wit, fail = run(name, inputs)
    assert fail is not None, name
    assert unsat(c, wit) != [], name
    return fail


def free_wires(c, wit):
    """IsZero / QuinSelector inverses of a zero input: circomlib's `inv <-- ...` is
    unconstrained when the input is 0 (out = 1 either way)."""
    free = set()
    for typ, err, n, dst, a, b, cc, extra in c.ops:
        if typ == circuit.OP_INV and wit[dst] == 0:
            free.add(dst)
        elif typ == circuit.OP_QUIN:
            free.update(i for i in range(dst + n, dst + 2 * n) if wit[i] == 0)
    return free


def single_signal_soundness(name, inputs, sample=None, seed=1):
    """Every computed signal is pinned by the constraints given the others: +1 on it
    breaks a constraint that mentions it."""
    c, prog, idx = built(name)
    wit, fail = wvm.evaluate(prog, [x % R for x in inputs])
    assert fail is None
    free = free_wires(c, wit)
    first = c.in_base + c.n_pub_in + c.n_prv_in
    wires = [k for k in list(range(1, c.in_base)) + list(range(first, c.n_wires)) if k not in free]
    if sample and len(wires) > sample:
        wires = random.Random(seed).sample(wires, sample)
    loose = []
    for k in wires:
        old = wit[k]
        wit[k] = (old + 1) % R
        if not _violated(c, wit, idx.get(k, ())):
            loose.append(k)
        wit[k] = old
    assert loose == [], (name, loose[:10])
    return len(wires)


def pad(a, n):  # test/helpers/cbor.js padArray
    return list(a) + [0] * (n - len(a))


def enc(x):
    return list(C.cbor(x))


def arr(*items):  # test/helpers/cbor.js encodeArray
    out = list(nzcp.cbor_head(4, len(items)))
    for it in items:
        out += it
    return out


# ---- test/cbor.js ---------------------------------------------------------------------
def test_get_type_get_x_exhaustive():                      # cbor.js:10-36
    for v in range(256):
        assert accept("getType_test", [v]) == [v >> 5]
        assert accept("getX_test", [v]) == [v & 31]


@pytest.mark.parametrize("n", [3, 4, 5])
def test_get_v(n):                                          # cbor.js:38-105
    for pos in range(n):
        assert accept(f"getV{n}_test", list(range(1, n + 1)) + [pos]) == [pos + 1]


def test_decode_uint23_accepts_and_rejects():              # cbor.js:108-127
    for v in range(256):
        if (v & 31) <= 23:
            assert accept("decodeUint32_test", [v]) == [v & 31]
        else:
            assert reject("decodeUint32_test", [v])[1] == nzcpgen.ERR_UINT23


@pytest.mark.parametrize("bs,v,want", [
    ([0, 0, 0, 0], 167, 7), ([0, 0, 0, 0], 168, 8), ([31, 0, 0, 0], 120, 31), ([38, 0, 0, 0], 120, 38),
    ([42, 69, 0, 0], 25, 10821), ([69, 42, 0, 0], 25, 17706), ([97, 218, 192, 48], 26, 1641726000),
    ([98, 150, 3, 64], 26, 1653998400)])
def test_decode_uint(bs, v, want):                          # cbor.js:129-179
    assert accept("decodeUint_test", [v] + bs + [0])[0] == want


def test_read_type():                                       # cbor.js:181-218
    for v in range(256):
        for bs, pos in (([0, 0, v], 2), ([0, v, 0], 1), ([v, 0, 0], 0)):
            assert accept("readType_test", bs + [pos]) == [pos + 1, v >> 5, v]


SCALARS = [enc("a" * n) for n in range(5)] + [enc(v) for v in range(24)] + [enc(0xFF), enc(0xFFFF)]


@pytest.mark.parametrize("name", ["skipValueScalar_test", "skipValue5_test"])
def test_skip_value_scalars(name):                          # cbor.js:221-302
    for cb in SCALARS:
        assert accept(name, pad(cb, 5) + [0]) == [len(cb)]
    cb = enc(0xFFFFFFFF)                                    # 5 bytes: fills the 5-byte buffer
    assert accept(name, pad(cb, 5) + [0]) == [len(cb)]


@pytest.mark.parametrize("items,name", [
    ([enc(23)] * 3, "skipValue5_test"), ([enc(23)] * 4, "skipValue5_test"),
    ([enc(0xFF)] * 2, "skipValue5_test"), ([enc(0xFFFF)], "skipValue5_test"),
    ([enc(0xFFFFFFFF)], "skipValue6_test"), ([enc("q")] * 2, "skipValue5_test"),
    ([enc("qwe")], "skipValue5_test"), ([enc("q"), enc(0xFF)], "skipValue5_test"),
    ([enc("q"), enc(23), enc(23)], "skipValue5_test")])
def test_skip_value_arrays(items, name):                    # cbor.js:305-368
    cb = arr(*items)
    n = 6 if name == "skipValue6_test" else 5
    assert accept(name, pad(cb, n) + [0]) == [len(cb)]
    assert nz.skip_value(pad(cb, n), 0, 4) == len(cb)      # the restatement agrees


def test_skip_value_array_edges():
    """An array longer than MaxArrayLen (QuinSelector index 4 of 4) is rejected by a
    constraint, as by the restatement. The empty array is accepted with nextPos 0, by the
    template as written: its index -1 passes QuinSelector's LessThan(3) (-1 + 8 - 4 = 3 fits
    in 4 bits) and selects nothing; the restatement agrees."""
    cb = [0x85, 1, 2, 3, 4]
    fail = reject("skipValue5_test", pad(cb, 5) + [0])
    with pytest.raises(nz.CircuitError) as e:
        nz.skip_value(pad(cb, 5), 0, 4)
    assert fail[1] == e.value.code == nzcpgen.ERR_SELECT
    assert accept("skipValue5_test", pad(arr(), 5) + [0]) == [0] == [nz.skip_value(pad(arr(), 5), 0, 4)]


def test_read_string_length():                             # cbor.js:370-384
    for n in range(5):
        assert accept("readStringLength_test", pad(enc("a" * n), 5) + [0]) == [n, 1]
    assert reject("readStringLength_test", pad(enc(7), 5) + [0])[1] == nzcpgen.ERR_NOT_STRING


def test_string_equals():                                   # cbor.js:386-407
    assert accept("stringEquals_test", pad(list(b"abcde"), 5) + [0, 5]) == [1]
    for n in range(6):
        assert accept("stringEquals_test", pad(list(b"b" * n), 5) + [0, n]) == [0]


def test_read_map_length():                                 # cbor.js:409-432
    maps = [{4: 5}, {4: 5, 5: 4}, {4: 5, 5: 4, 7: 3}]
    for want, m in enumerate(maps, 1):
        assert accept("readMapLength_test", [0] + pad(enc(m), 7)) == [want, 1]
    assert reject("readMapLength_test", [0] + pad(enc([1]), 7))[1] == nzcpgen.ERR_NOT_MAP


@pytest.mark.parametrize("s", ["", "ab", "abcd"])
def test_copy_string(s):                                    # cbor.js:436-477
    out = accept("copyString_test", pad(enc(s), 5) + [0])
    assert out == pad(list(s.encode()), 4) + [len(s) + 1, len(s)]


# ---- test/quinSelector.js -------------------------------------------------------------
def test_quin_selector_kats():                              # quinSelector.js:22-61
    assert accept("quinSelector0_test", [R - 1]) == [0]     # index -1, no choices
    for n in range(1, 6):
        for index in range(n):
            assert accept(f"quinSelector{n}_test", list(range(1, n + 1)) + [index]) == [index + 1]


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5])
def test_quin_selector_rejects_index_n(n):                 # quinSelector.js:63-87
    assert reject(f"quinSelector{n}_test", list(range(1, n + 1)) + [n])[1] == nzcpgen.ERR_SELECT


# ---- test/nzcp.js: the template mains on whole passes ----------------------------------
def _bytes_of(tbs: bytes, n: int):
    return list((tbs + bytes(n))[:n])


PASSES = {
    # name: (ToBeSigned, max bytes, claims position, vcPos KAT, cred-subj position KAT)
    "example": (C.example_tbs(), 314, 28, 76, 246),                 # test/nzcp.js:100,164
    "live": (C.live_tbs(), 351, 31, 80, 250),                       # test/nzcp.js:117,207
}


@pytest.mark.parametrize("which", ["example", "live"])
def test_find_cwt_claims(which):                            # test/nzcp.js:82-143
    tbs, n, pos, vc_pos, _ = PASSES[which]
    out = accept(f"findCWTClaims_{which}Test", [5] + _bytes_of(tbs, n) + [pos])
    assert out == [vc_pos, nzcp.EXAMPLE_EXP]
    assert list(nz.find_cwt_claims(_bytes_of(tbs, n), pos, 5, 0, 4)) == out


@pytest.mark.parametrize("which", ["example", "live"])
def test_find_cred_subj(which):                             # test/nzcp.js:146-215
    tbs, n, _, vc_pos, cs_pos = PASSES[which]
    out = accept(f"findCredSubj_{which}Test", [4] + _bytes_of(tbs, n) + [vc_pos + 1])
    assert out == [cs_pos]
    assert nz.find_cred_subj(_bytes_of(tbs, n), vc_pos + 1, 4, 2, 4) == cs_pos


@pytest.mark.parametrize("which,max_buf", [("example", 32), ("live", 64)])
def test_read_cred_subj(which, max_buf):                    # test/nzcp.js:217-285
    tbs, n, _, _, cs_pos = PASSES[which]
    out = accept(f"readCredSubj_{which}Test", [3] + _bytes_of(tbs, n) + [cs_pos + 1])
    given, family, dob = b"Jack", b"Sparrow", b"1960-04-16"   # the MoH example subject
    want = []
    for s in (given, family, dob):
        want += pad(list(s), max_buf) + [len(s)]
    assert out == want
    # mapLen must be exactly 3 (hardcore_assert, nzcptpl.circom:261)
    reject(f"readCredSubj_{which}Test", [4] + _bytes_of(tbs, n) + [cs_pos + 1])


@pytest.mark.parametrize("names", [("Jack", "Sparrow", "1960-04-16"), ("Jo", "Bloggs", "1999-12-31"),
                                   ("A" * 21, "B" * 21, "1960-04-16")])
def test_construct_nullifier(names):                        # test/nzcp.js:287-331
    g, f, d = (s.encode() for s in names)
    ins = pad(list(g), 64) + [len(g)] + pad(list(f), 64) + [len(f)] + pad(list(d), 64) + [len(d)]
    out = accept("constructNullifier_test", ins)
    want = b",".join((g, f, d))
    assert out == pad(list(want), 64) + [len(want)]


# ---- soundness probes ------------------------------------------------------------------
@pytest.mark.parametrize("name,inputs", [
    ("getType_test", [0xA5]), ("decodeUint32_test", [0x37]), ("decodeUint_test", [26, 97, 218, 192, 48, 0]),
    ("readType_test", [0, 0x63, 0, 1]), ("skipValueScalar_test", pad(enc("abc"), 5) + [0]),
    ("skipValue5_test", pad(arr(enc("q"), enc(23), enc(23)), 5) + [0]),
    ("stringEquals_test", pad(list(b"abcde"), 5) + [0, 5]), ("readStringLength_test", pad(enc("ab"), 5) + [0]),
    ("readMapLength_test", [0] + pad(enc({4: 5, 5: 4}), 7)), ("copyString_test", pad(enc("abcd"), 5) + [0]),
    ("quinSelector5_test", [1, 2, 3, 4, 5, 3])])
def test_every_signal_is_constrained(name, inputs):
    assert single_signal_soundness(name, inputs) > 0


@pytest.mark.parametrize("which", ["example", "live"])
def test_every_signal_is_constrained_on_passes(which):
    """The same probe on the pass-sized mains (a seeded sample of their signals)."""
    tbs, n, pos, vc_pos, cs_pos = PASSES[which]
    assert single_signal_soundness(f"findCWTClaims_{which}Test", [5] + _bytes_of(tbs, n) + [pos], sample=1500)
    assert single_signal_soundness(f"readCredSubj_{which}Test", [3] + _bytes_of(tbs, n) + [cs_pos + 1],
                                   sample=1500)


def test_tampered_selectors_are_rejected():
    """A prover that makes QuinSelector return another element, or flips an IsZero output
    (and then recomputes every downstream signal the way the calculator would) still
    breaks a constraint: the selector's eq/inv rows pin the selected index."""
    name = "quinSelector5_test"
    c, prog, _ = built(name)
    wit, fail = wvm.evaluate(prog, [1, 2, 3, 4, 5, 2])
    assert fail is None and wit[1] == 3
    (typ, err, n, base, a, b, cc, extra), = [op for op in c.ops if op[0] == circuit.OP_QUIN]
    forged = list(wit)
    for i in range(n):                       # eq one-hot at index 4 instead of 2
        forged[base + i] = 1 if i == 4 else 0
    s = 0
    for i in range(n):                       # running sums recomputed for the forged eq
        s = (s + forged[base + i] * forged[extra[0] + i]) % R
        forged[base + 2 * n + i] = s
    forged[1] = s
    assert forged[1] == 5 and unsat(c, forged) != []
    # IsZero flipped: ReadMapLength's type check on a string, out forced to "is a map"
    c, prog, _ = built("stringEquals_test")
    wit, fail = wvm.evaluate(prog, pad(list(b"abcdx"), 5) + [0, 5])
    assert fail is None and wit[1] == 0
    for typ, err, n_, dst, a, b, cc, extra in c.ops:
        if typ == circuit.OP_INV and wit[dst]:
            forged = list(wit)
            out_wire = dst + 1                # IsZero: inv, then out = -x inv + 1 (Circuit.is_zero)
            forged[out_wire] = (1 - forged[out_wire]) % R
            assert unsat(c, forged) != []
