"""CPU restatement of the nzcp circuit (oracle/nzcp_circuit.py) pinned by the
reference's own known-answer tests: the CBOR gadget KATs of test/cbor.js, the
QuinSelector KATs of test/quinSelector.js, the example-pass checks of test/nzcp.js
and test/utils.js, and SURVEY.md §8c's public signals for the example pass."""
import hashlib
import json
import os

import pytest

import nzcp_cases as C
from oracle import nzcp_circuit as nz
from oracle.nzcp_circuit import CircuitError

GOLD = os.path.join(os.path.dirname(__file__), "golden", "nzcp_cases.json")


def pad(a, n):  # test/helpers/cbor.js padArray
    return list(a) + [0] * (n - len(a))


def enc_int(v):  # test/helpers/cbor.js encodeInt
    return list(C.cbor(v))


def enc_str(s):
    return list(C.cbor(s))


# ---- test/cbor.js -----------------------------------------------------------------
def test_get_type_get_x_exhaustive():  # test/cbor.js:10-36
    for v in range(256):
        assert nz.get_type(v) == v >> 5
        assert nz.get_x(v) == v & 31


@pytest.mark.parametrize("n", [3, 4, 5])
def test_get_v(n):  # test/cbor.js:38-110
    bs = list(range(1, n + 1))
    for pos in range(n):
        assert nz.get_v(bs, pos) == pos + 1


def test_decode_uint23_accepts_and_rejects():  # test/cbor.js:113-131
    for v in range(256):
        if (v & 31) <= 23:
            assert nz.decode_uint23(v) == v & 31
        else:
            with pytest.raises(CircuitError):
                nz.decode_uint23(v)


@pytest.mark.parametrize("bs,v,want", [
    ([0, 0, 0, 0], 167, 7), ([0, 0, 0, 0], 168, 8), ([31, 0, 0, 0], 120, 31), ([38, 0, 0, 0], 120, 38),
    ([42, 69, 0, 0], 25, 10821), ([69, 42, 0, 0], 25, 17706), ([97, 218, 192, 48], 26, 1641726000),
    ([98, 150, 3, 64], 26, 1653998400)])
def test_decode_uint(bs, v, want):  # test/cbor.js:133-183
    assert nz.decode_uint(bs, 0, v)[0] == want


def test_read_type():  # test/cbor.js:185-217
    for v in range(256):
        for bs, pos in (([0, 0, v], 2), ([0, v, 0], 1), ([v, 0, 0], 0)):
            assert nz.read_type(bs, pos) == (pos + 1, v >> 5, v)


def test_skip_value_scalar_and_skip_value():  # test/cbor.js:220-315
    for n in range(5):
        cb = enc_str("a" * n)
        assert nz.skip_value_scalar(pad(cb, 5), 0) == n + 1
        assert nz.skip_value(pad(cb, 5), 0, 4) == n + 1
    for v in list(range(24)) + [0xFF, 0xFFFF]:
        cb = enc_int(v)
        assert nz.skip_value_scalar(pad(cb, 5), 0) == len(cb)
        assert nz.skip_value(pad(cb, 5), 0, 4) == len(cb)
    cb = enc_int(0xFFFFFFFF)
    assert nz.skip_value_scalar(pad(cb, 5), 0) == len(cb)
    assert nz.skip_value(pad(cb, 5), 0, 4) == len(cb)


@pytest.mark.parametrize("items,n", [
    ([23, 23, 23], 5), ([23, 23, 23, 23], 5), ([0xFF, 0xFF], 5), ([0xFFFF], 5), ([0xFFFFFFFF], 6),
    (["q", "q"], 5), (["qwe"], 5), (["q", 0xFF], 5), (["q", 23, 23], 5)])
def test_skip_value_array(items, n):  # test/cbor.js:318-386 (SkipValue(5|6, 4))
    cb = list(C.cbor(items))
    assert nz.skip_value(pad(cb, n), 0, 4) == len(cb)


def test_read_string_length():  # test/cbor.js:388-401
    for n in range(5):
        assert nz.read_string_length(pad(enc_str("a" * n), 5), 0) == (n, 1)


def test_string_equals():  # test/cbor.js:403-424 (StringEquals(5, "abcde", 5))
    assert nz.string_equals(list(b"abcde"), 0, 5, b"abcde") == 1
    for n in range(6):
        assert nz.string_equals(pad(list(b"b" * n), 5), 0, n, b"abcde") == 0


@pytest.mark.parametrize("m", [{4: 5}, {4: 5, 5: 4}, {4: 5, 5: 4, 7: 3}])
def test_read_map_length(m):  # test/cbor.js:426-449 (ReadMapLength(7))
    assert nz.read_map_length(pad(list(C.cbor(m)), 7), 0)[0] == len(m)


@pytest.mark.parametrize("s", ["", "ab", "abcd"])
def test_copy_string(s):  # test/cbor.js:453-476 (CopyString(5, 4))
    out, nxt, ln = nz.copy_string(pad(enc_str(s), 5), 0, 4)
    assert out == pad(list(s.encode()), 4) and nxt == len(s) + 1 and ln == len(s)


# ---- test/quinSelector.js -------------------------------------------------------------
@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 5])
def test_quin_selector(n):  # test/quinSelector.js:23-86
    arr = list(range(1, n + 1))
    for i in range(n):
        assert nz.quin_selector(arr, i) == i + 1
    if n == 0:
        assert nz.quin_selector(arr, 0) == 0
    else:
        with pytest.raises(CircuitError) as e:
            nz.quin_selector(arr, n)
        assert e.value.code == nz.ERR_SELECT


def test_log2():  # log2.circom:5-12 (test/log2.js)
    assert [nz.log2(x) for x in (0, 1, 2, 3, 4, 63, 64, 351, 352)] == [-1, 0, 1, 1, 2, 5, 6, 8, 8]


# ---- test/nzcp.js / test/utils.js ------------------------------------------------------
def test_example_tbs_sha256_kat():  # test/utils.js:16-20
    assert hashlib.sha256(C.example_tbs()).hexdigest() == \
        "271ce33d671a2d3b816d788135f4343e14bc66802f8cd841faac939e8c11f3ee"


def test_find_cwt_claims_example_and_live():  # test/nzcp.js:78-130
    bs = list(C.example_tbs())
    assert nz.find_cwt_claims(bs, 28, 5, 0, 4) == (76, C.EXAMPLE_EXP)
    bs = pad(list(C.live_tbs()), 351)
    assert nz.find_cwt_claims(bs, 31, 5, 0, 4) == (80, C.EXAMPLE_EXP)


def test_read_cred_subj_example_and_live():  # test/nzcp.js:186-247
    bs = list(C.example_tbs())
    g, gl, f, fl, d, dl = nz.read_cred_subj(bs, 247, 3, 32)
    assert (g, gl) == (pad(list(b"Jack"), 32), 4)
    assert (f, fl) == (pad(list(b"Sparrow"), 32), 7)
    assert (d, dl) == (pad(list(b"1960-04-16"), 32), 10)
    bs = pad(list(C.live_tbs()), 351)
    assert nz.read_cred_subj(bs, 251, 3, 64)[0] == pad(list(b"Jack"), 64)


def test_construct_nullifier():  # test/nzcp.js:249-281
    res, ln = nz.construct_nullifier(pad(list(b"Jack"), 64), 4, pad(list(b"Sparrow"), 64), 7,
                                     pad(list(b"1960-04-16"), 64), 10)
    assert res == pad(list(b"Jack,Sparrow,1960-04-16"), 64) and ln == 23


def test_example_pass_public_signals():  # test/nzcp.js:33-69,341-351; SURVEY.md §8c
    bits, ln, data = nz.circuit_input(C.example_tbs(), C.DATA_1_20, 314)
    w = nz.nzcp_pub_identity(bits, ln, data, **nz.EXAMPLE_PARAMS)
    assert w.status == nz.OK
    assert (w.vc_pos, w.exp) == (76, 1951416330)
    assert w.nullifier.rstrip(b"\0") == b"Jack,Sparrow,1960-04-16"
    assert w.nullifier_sha512[:32].hex() == "04ca63f107c06816c14bf8f3f93b6b4b3ea3a1d17240d25448062c6e6d6a92bd"
    assert w.out == [
        8464235439336389695359576364537904521787463454426143836621154307990710930,
        334204042160295982690797293769892102755483197293558786265320143920457223185,
        430989588176824417852954207888075491695208395262355815151652761069951123456]
    assert w.out == nz.expected_public_signals(C.example_tbs(), b"Jack,Sparrow,1960-04-16", C.EXAMPLE_EXP,
                                               C.DATA_1_20)


def test_live_shaped_pass_matches_the_tests_decode():  # test/nzcp.js:33-69 with the live circuit
    for names in (("Jack", "Sparrow", "1960-04-16"), ("Jo", "Bloggs", "1999-12-31")):
        tbs = C.live_tbs(subject=C.credential_subject(*names))
        data = bytes(range(50, 70))
        bits, ln, d = nz.circuit_input(tbs, data, 351)
        w = nz.nzcp_pub_identity(bits, ln, d, **nz.LIVE_PARAMS)
        assert w.status == nz.OK and w.vc_pos == 80
        assert w.out == nz.expected_public_signals(tbs, ",".join(names).encode(), C.EXAMPLE_EXP, data)


def test_golden_fixture_is_current():
    with open(GOLD) as f:
        gold = json.load(f)
    cases = C.all_cases()
    assert [c["name"] for c in cases] == [c["name"] for c in gold["cases"]]
    assert cases == gold["cases"]
    assert [C.oracle_record(c) for c in gold["cases"]] == gold["expected"]
    statuses = {r["status"] for r in gold["expected"]}
    assert statuses >= {nz.OK, nz.ERR_BIT, nz.ERR_LEN, nz.ERR_RANGE, nz.ERR_SELECT, nz.ERR_NOT_MAP,
                        nz.ERR_UINT23, nz.ERR_NOT_STRING, nz.ERR_UNPINNED}


def test_free_public_synth_accepts_any_public_values():
    """NZCB_SYNTH_FREE_PUBLIC circuits stay satisfied when witness[1..3] are replaced
    by nzcp outputs (the fullProve stand-in of bench.py): oracle prove + trapdoor verify."""
    from oracle import plonk, synth
    c = synth.synth_circuit(6, 3, 5, seed=11, free_public=True)
    zk = plonk.setup(c, 4321)
    bits, ln, data = nz.circuit_input(C.live_tbs(), C.DATA_1_20, 351)
    out = nz.nzcp_pub_identity(bits, ln, data, **nz.LIVE_PARAMS).out
    wit = list(c["witness"])
    wit[1:4] = out
    proof, pub = plonk.prove(zk, wit, synth.fixed_blindings())
    assert pub == out
    assert plonk.verify_with_trapdoor(zk, pub, proof, 4321)
    # the default family wires the public signals into later gates: replacing them breaks it
    c2 = synth.synth_circuit(6, 3, 5, seed=11)
    assert any(s in (1, 2, 3) for g in c2["constraints"][3:] for s in g[:3])
    assert not any(s in (1, 2, 3) for g in c["constraints"][3:] for s in g[:3])


def test_bench_passes_are_valid_and_distinct():
    """bench.py's per-proof passes: the restatement accepts them with distinct outputs."""
    import bench
    from oracle.bn254 import R_MOD  # noqa: F401
    raw = bench.pass_inputs(range(3))
    per = (351 * 8 + 161) * 32
    assert len(raw) == 3 * per
    outs = []
    for i in range(3):
        sig = [int.from_bytes(raw[i * per + 32 * k:i * per + 32 * k + 32], "little") for k in range(351 * 8 + 161)]
        w = nz.nzcp_pub_identity(sig[:2808], sig[2808], sig[2809:], **nz.LIVE_PARAMS)
        assert w.status == nz.OK and w.vc_pos == 80
        outs.append(tuple(w.out))
    assert len(set(outs)) == 3
