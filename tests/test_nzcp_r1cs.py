"""The nzcp_live circuit as an r1cs + witness program (nzcb/circuit.py, nzcb/nzcpgen.py),
checked on the CPU:

* gadgets: the SHA-512 (64-byte message) and variable-length SHA-256 gadgets give
  hashlib's digests and satisfy their constraints, at every length class;
* NZCPPubIdentity(1, 351, 0, 4, 2, 4): the CPU evaluation of the witness program
  (oracle/wvm.py) satisfies every r1cs constraint, every wire is written by exactly one
  operation, the public outputs equal the CPU restatement oracle/nzcp_circuit.py (pinned
  by the reference's test vectors), and failing passes fail with the restatement's status;
* size: snarkjs plonk setup makes 2^20 < gates <= 2^21 of it (the ptau-21 domain of
  /root/reference/Makefile:60); r1cs write/read round trip on a gadget circuit.

Parity against circom's own r1cs / wasm is unpinned (nzcb/nzcpgen.py docstring)."""
import hashlib
import random

import pytest

import nzcp_cases as C
from nzcb import circuit, nzcpgen
from nzcb.circuit import Circuit, w
from oracle import nzcp_circuit as nz
from oracle import r1cs as r1cs_oracle
from oracle import wvm

R = circuit.R


def _unsat(c: Circuit, wit, limit=3):
    bad = []
    for k, (A, B, Cc) in enumerate(c.constraints):
        a = sum(v * wit[i] for i, v in A.items()) % R
        b = sum(v * wit[i] for i, v in B.items()) % R
        cc = sum(v * wit[i] for i, v in Cc.items()) % R
        if (a * b - cc) % R:
            bad.append(k)
            if len(bad) >= limit:
                break
    return bad


def _written(c: Circuit):
    """wire -> number of ops writing it (inputs and wire 0 count once)."""
    cnt = [0] * c.n_wires
    cnt[0] = 1
    for i in range(c.in_base, c.in_base + c.n_pub_in + c.n_prv_in):
        cnt[i] += 1
    for typ, err, n, dst, a, b, cc, extra in c.ops:
        if typ == circuit.OP_QUIN:
            width = 2 * n + extra[1]
        elif typ in (circuit.OP_SHA256, circuit.OP_SHA512):
            width = circuit.sha_block_layout(circuit.SHA256_SPEC if typ == circuit.OP_SHA256
                                             else circuit.SHA512_SPEC)["size"]
        elif typ == circuit.OP_BITS:
            width = n
        elif typ == circuit.OP_CHECK:
            width = 0
        else:
            width = 1
        for k in range(dst, dst + width):
            cnt[k] += 1
    return cnt


def _bits_lsb_bytes(data: bytes):
    return [(b >> j) & 1 for b in data for j in range(8)]


def test_sha512_gadget_matches_hashlib():
    c = Circuit(0, 0, 512)
    out = nzcpgen.sha512_64(c, c.in_base)
    prog = c.write_program()
    rng = random.Random(5)
    for msg in (bytes(64), bytes(range(64)), bytes(rng.randrange(256) for _ in range(64))):
        wit, fail = wvm.evaluate(prog, _bits_lsb_bytes(msg))
        assert fail is None and _unsat(c, wit) == []
        digest = [sum(v * wit[i] for i, v in bit.items()) % R for bit in out]
        want = hashlib.sha512(msg).digest()
        assert digest == [(want[k // 8] >> (7 - k % 8)) & 1 for k in range(512)]
    assert _written(c)[1:] == [1] * (c.n_wires - 1)


@pytest.mark.parametrize("length", [0, 1, 31, 55, 56, 63, 64, 100, 119])
def test_sha256_var_gadget_matches_hashlib(length):
    max_bytes = 120
    c = Circuit(0, 0, 8 * max_bytes + 1)
    bits = [w(c.in_base + i) for i in range(8 * max_bytes)]
    out = nzcpgen.sha256_var(c, bits, w(c.in_base + 8 * max_bytes), 1)
    prog = c.write_program()
    rng = random.Random(length)
    msg = bytes(rng.randrange(256) for _ in range(length))
    fitted = msg + bytes(max_bytes - length)
    inp = [(b >> (7 - j)) & 1 for b in fitted for j in range(8)] + [length]
    wit, fail = wvm.evaluate(prog, inp)
    assert fail is None and _unsat(c, wit) == []
    digest = [sum(v * wit[i] for i, v in bit.items()) % R for bit in out]
    want = hashlib.sha256(msg).digest()
    assert digest == [(want[k // 8] >> (7 - k % 8)) & 1 for k in range(256)]
    # bytes past the length are masked: garbage there does not change the digest
    noisy = fitted[:length] + bytes(rng.randrange(256) for _ in range(max_bytes - length))
    inp2 = [(b >> (7 - j)) & 1 for b in noisy for j in range(8)] + [length]
    wit2, _ = wvm.evaluate(prog, inp2)
    assert [sum(v * wit2[i] for i, v in bit.items()) % R for bit in out] == digest


def test_r1cs_file_round_trip():
    c = Circuit(0, 0, 512)
    nzcpgen.sha512_64(c, c.in_base)
    rd = r1cs_oracle.read_r1cs(c.write_r1cs())
    assert rd["prime"] == R and rd["nWires"] == c.n_wires and rd["nPrvInputs"] == 512
    assert len(rd["constraints"]) == len(c.constraints)
    for (A, B, Cc), (a, b, cc) in zip(c.constraints[::997], rd["constraints"][::997]):
        assert dict(a) == A and dict(b) == B and dict(cc) == Cc


@pytest.fixture(scope="module")
def live():
    c = nzcpgen.nzcp_pub_identity(**nzcpgen.LIVE)
    return c, c.write_program()


def test_live_circuit_size(live):
    c, _ = live
    gates = circuit.plonk_gate_count(c)
    assert (1 << 20) < gates <= (1 << 21)
    assert c.n_out == 3 and c.n_pub_in == 0 and c.n_prv_in == 351 * 8 + 1 + 160
    assert _written(c) == [1] * c.n_wires


def _case_inputs(case):
    bits, ln, data = C.case_signals(case)
    return bits + [ln] + data


@pytest.mark.parametrize("name,make", [
    ("live", lambda: C.case("live", nz.LIVE_PARAMS, C.live_tbs(), data=bytes(range(1, 21)))),
    ("jo", lambda: C.case("jo", nz.LIVE_PARAMS, C.live_tbs(subject=C.credential_subject("Jo", "Bloggs", "1999-12-31")),
                          data=bytes(range(7, 27)))),
    ("long-names", lambda: C.case("long", nz.LIVE_PARAMS, C.live_tbs(
        subject=C.credential_subject("A" * 21, "B" * 21, "1960-04-16")))),
])
def test_live_witness_satisfies_r1cs_and_matches_oracle(live, name, make):
    c, prog = live
    case = make()
    wit, fail = wvm.evaluate(prog, _case_inputs(case))
    exp = C.oracle_record(case)
    assert exp["status"] == 0 and fail is None
    assert wit[1:4] == [int(v) for v in exp["out"]]
    assert _unsat(c, wit) == []


@pytest.mark.parametrize("kind", ["len", "bit", "map"])
def test_live_failing_passes(live, kind):
    """Rejected passes: the witness program fails with the restatement's status code."""
    c, prog = live
    if kind == "len":
        case = C.case("len", nz.LIVE_PARAMS, C.live_tbs(), length=352)
    elif kind == "bit":
        case = C.case("bit", nz.LIVE_PARAMS, C.live_tbs(), bit_overrides={17: 2})
    else:
        tbs = bytearray(C.live_tbs())
        tbs[30] = 0x61          # claims at byte 30 are not a map
        case = C.case("map", nz.LIVE_PARAMS, bytes(tbs))
    exp = C.oracle_record(case)
    wit, fail = wvm.evaluate(prog, _case_inputs(case))
    assert exp["status"] != 0 and fail is not None
    assert fail[1] == exp["status"]
    # soundness: the witness carried past the failure is not a satisfying
    # assignment; the rejection is a constraint of the r1cs, not only a calculator check
    assert _unsat(c, wit) != []


def test_live_every_sampled_signal_is_constrained(live):
    """Soundness probe on NZCPPubIdentity(1, 351, 0, 4, 2, 4): for a seeded sample of 4000
    computed signals of a valid pass's witness (SHA-256/512 rounds, CBOR parsing,
    QuinSelectors, nullifier bytes alike), +1 on the signal breaks a constraint that
    mentions it. IsZero / QuinSelector inverses of zero inputs are circomlib's free
    signals and are skipped."""
    c, prog = live
    case = C.case("live", nz.LIVE_PARAMS, C.live_tbs(), data=bytes(range(1, 21)))
    wit, fail = wvm.evaluate(prog, _case_inputs(case))
    assert fail is None
    free = set()
    for typ, err, n, dst, a, b, cc, extra in c.ops:
        if typ == circuit.OP_INV and wit[dst] == 0:
            free.add(dst)
        elif typ == circuit.OP_QUIN:
            free.update(i for i in range(dst + n, dst + 2 * n) if wit[i] == 0)
    first = c.in_base + c.n_pub_in + c.n_prv_in
    cand = [k for k in list(range(1, c.in_base)) + list(range(first, c.n_wires)) if k not in free]
    sample = set(random.Random(0x50554E44).sample(cand, 4000))
    touching = {}
    for k, cons in enumerate(c.constraints):
        for part in cons:
            for wire in part:
                if wire in sample:
                    touching.setdefault(wire, []).append(k)
    loose = []
    for k in sorted(sample):
        old = wit[k]
        wit[k] = (old + 1) % R
        ok = False
        for j in touching.get(k, ()):
            A, B, Cc = c.constraints[j]
            a = sum(v * wit[i] for i, v in A.items()) % R
            b = sum(v * wit[i] for i, v in B.items()) % R
            cv = sum(v * wit[i] for i, v in Cc.items()) % R
            if (a * b - cv) % R:
                ok = True
                break
        wit[k] = old
        if not ok:
            loose.append(k)
    assert loose == []
