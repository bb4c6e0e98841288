"""nzcp witness kernel (csrc/nzcp.hip) on the GPU vs the CPU restatement
(oracle/nzcp_circuit.py): every committed golden case bit-exact (public signals,
digests, nullifier, lengths, status and detail), a large batch of distinct passes,
and the device path that writes the public signals into prover witnesses."""
import ctypes
import json
import os
import random

import pytest

import nzcp_cases as C
from oracle import nzcp_circuit as nz

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "nzcp_cases.json")


@pytest.fixture(scope="module")
def nzcb_mod():
    import nzcb
    if nzcb.device_count() < 1:
        pytest.fail("GPU test requested but no HIP device is visible")
    return nzcb


def _run(nzcb, cases, params):
    inputs = b"".join(C.case_input_bytes(c) for c in cases)
    return [C.gpu_record_json(r) for r in nzcb.nzcp_witness(inputs, len(cases), params)]


def test_golden_cases_bit_exact(nzcb_mod):
    with open(GOLD) as f:
        gold = json.load(f)
    groups = {}
    for c, e in zip(gold["cases"], gold["expected"]):
        groups.setdefault(json.dumps(c["params"], sort_keys=True), []).append((c, e))
    n = 0
    for key, items in groups.items():
        got = _run(nzcb_mod, [c for c, _ in items], json.loads(key))
        for (c, e), g in zip(items, got):
            assert g == e, c["name"]
            n += 1
    assert n == len(gold["cases"])


def test_example_pass_kat(nzcb_mod):  # SURVEY.md §8c, test/nzcp.js:33-69
    c = C.case("example", nz.EXAMPLE_PARAMS, C.example_tbs())
    (r,) = nzcb_mod.nzcp_witness(C.case_input_bytes(c), 1, nzcb_mod.NZCP_EXAMPLE)
    assert r["status"] == 0 and r["vc_pos"] == 76
    assert r["tbs_sha256"].hex() == "271ce33d671a2d3b816d788135f4343e14bc66802f8cd841faac939e8c11f3ee"
    assert r["out"] == [
        8464235439336389695359576364537904521787463454426143836621154307990710930,
        334204042160295982690797293769892102755483197293558786265320143920457223185,
        430989588176824417852954207888075491695208395262355815151652761069951123456]


def test_large_batch_distinct_passes(nzcb_mod):
    """512 passes (the configs[3] batch size) with distinct names and data."""
    rng = random.Random(7)
    cases = []
    for i in range(512):
        g = "".join(rng.choice("abcdefghij") for _ in range(rng.randrange(1, 21)))
        f = "".join(rng.choice("klmnopqrst") for _ in range(rng.randrange(1, 21)))
        d = f"19{rng.randrange(10, 99)}-0{rng.randrange(1, 9)}-1{rng.randrange(0, 9)}"
        data = bytes(rng.randrange(256) for _ in range(20))
        cases.append(C.case(f"p{i}", nz.LIVE_PARAMS, C.live_tbs(subject=C.credential_subject(g, f, d)), data=data))
    got = _run(nzcb_mod, cases, nz.LIVE_PARAMS)
    assert all(g["status"] == 0 for g in got)
    assert len({tuple(g["out"]) for g in got}) == 512
    for i in range(0, 512, 37):
        assert got[i] == C.oracle_record(cases[i])


def test_device_path_writes_witness_publics(nzcb_mod):
    nzcb = nzcb_mod
    cases = [C.case(f"w{i}", nz.LIVE_PARAMS, C.live_tbs(), data=bytes([i]) * 20) for i in range(5)]
    cases.append(C.case("bad", nz.LIVE_PARAMS, C.live_tbs(), length=400))
    inputs = b"".join(C.case_input_bytes(c) for c in cases)
    n_wit, count = 16, len(cases)
    stride = n_wit * 32
    sentinel = bytes([0xA5]) * (stride * count)
    d_in = nzcb.dev_alloc(len(inputs))
    d_wit = nzcb.dev_alloc(len(sentinel))
    rec_size = ctypes.sizeof(nzcb.NzcpRecord)
    d_rec = nzcb.dev_alloc(rec_size * count)
    try:
        nzcb.h2d(d_in, inputs)
        nzcb.h2d(d_wit, sentinel)
        nzcb.nzcp_witness_dev(d_in, count, nzcb.NZCP_LIVE, dev_records=d_rec, dev_witness=d_wit,
                              witness_stride=stride)
        wit = nzcb.d2h(d_wit, len(sentinel))
        recs = nzcb.nzcp_records_from_bytes(nzcb.d2h(d_rec, rec_size * count), count)
    finally:
        for p in (d_in, d_wit, d_rec):
            nzcb.dev_free(p)
    for i, c in enumerate(cases):
        w = wit[i * stride:(i + 1) * stride]
        exp = C.oracle_record(c)
        assert C.gpu_record_json(recs[i]) == exp
        if exp["status"] == 0:
            assert [int.from_bytes(w[32 * k:32 * k + 32], "little") for k in (1, 2, 3)] == \
                [int(v) for v in exp["out"]]
            assert w[:32] == sentinel[:32] and w[128:] == sentinel[128:stride]  # only witness[1..3] written
        else:
            assert w == sentinel[:stride]


def test_bad_params_rejected(nzcb_mod):
    with pytest.raises(nzcb_mod.NzcbError):
        nzcb_mod.nzcp_witness(b"", 0, dict(is_live=1, max_tbs_bytes=600, max_array_len_vc=0, max_map_len_vc=4))


@pytest.mark.parametrize("power,nin,seed", [(6, 4, 21), (8, 8, 22)])
def test_free_public_synth_bytes(nzcb_mod, power, nin, seed):
    from oracle import binfmt, plonk, synth
    zkey, wtns = nzcb_mod.synth_setup(power, 3, nin, seed, 0, 555, free_public=True)
    c = synth.synth_circuit(power, 3, nin, seed=seed, free_public=True)
    assert wtns == binfmt.write_wtns(c["witness"])
    assert zkey == binfmt.write_zkey(plonk.setup(c, 555))


def test_full_prove_pipeline_bit_exact(nzcb_mod):
    """fullProve on device: nzcp witness kernel -> witness[1..3] in HBM -> prove_batch.
    Proofs bit-exact against the C oracle prover on the same witness (publics replaced
    by the CPU restatement's outputs), publics equal the restatement's, pairing-verified."""
    from oracle import cbind, synth
    nzcb = nzcb_mod
    zkey, wtns = nzcb.synth_setup(12, 3, 2970, 0x6E7A6362, 0, 0x6E7A6362746175, free_public=True)
    nwit = (len(wtns) - 76) // 32
    base = wtns[76:76 + 32 * nwit]
    ctx = nzcb.ProverContext(zkey)
    ctx.set_lanes(2)
    prover = nzcb.NzcpProver(ctx, base)
    cases = [C.case(f"p{i}", nz.LIVE_PARAMS, C.live_tbs(subject=C.credential_subject(g, f, "1960-04-16")),
                    data=bytes([i + 1]) * 20)
             for i, (g, f) in enumerate((("Jack", "Sparrow"), ("Jo", "Bloggs"), ("Ana", "Te Whare")))]
    bl = b"".join(x.to_bytes(32, "little") for x in synth.fixed_blindings())
    try:
        res, recs = prover.full_prove(b"".join(C.case_input_bytes(c) for c in cases), [bl] * 3)
        with pytest.raises(nzcb.NzcbError):
            prover.full_prove(C.case_input_bytes(C.case("bad", nz.LIVE_PARAMS, C.live_tbs(), length=360)))
    finally:
        prover.close()
        ctx.close()
    for c, (proof, pub), r in zip(cases, res, recs):
        exp = [int(v) for v in C.oracle_record(c)["out"]]
        assert [int.from_bytes(pub[32 * k:32 * k + 32], "little") for k in range(3)] == exp == r["out"]
        assert nzcb.verify(ctx.vk, proof, pub)
        w = bytearray(wtns)
        for k in range(3):
            w[76 + 32 * (1 + k):76 + 32 * (2 + k)] = exp[k].to_bytes(32, "little")
        ref_proof, ref_pub, _ = cbind.prove(zkey, bytes(w), bl, npub=3)
        assert proof == ref_proof and pub == ref_pub[:96]
