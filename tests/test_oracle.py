"""CPU oracle self-checks (no GPU): constants, keccak, curve, NTT, MSM, PLONK
setup/prove/verify, and the committed golden fixtures (tests/golden/)."""
import json
import os
import random

import pytest

from oracle import binfmt, bn254 as bn, plonk, synth
from oracle.keccak import keccak256
from oracle.bn254 import P_MOD, R_MOD

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_constants_match_survey():
    # SURVEY.md §8 constants table
    assert bn.FR_W[21] == 13536764371732269273912573961853310557438878140379554347802702086337840854307
    assert bn.FR_W[23] == 934650972362265999028062457054462628285482693704334323590406443310927365533
    assert bn.FR_W[28] == 19103219067921713944291392827692070036145651957329286315305642004821462161904
    assert pow(bn.FR_W[28], 1 << 27, R_MOD) == R_MOD - 1
    assert pow(bn.FR_W[28], 1 << 28, R_MOD) == 1


def test_keccak_known_answers():
    assert keccak256(b"").hex() == "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470"
    assert keccak256(b"abc").hex() == "4e03657aea45a94fc7d47ba826c8d667c0d1e6e33a64a036ec44f58fa12d6c45"
    # multi-block input (> 136-byte rate) and exact-rate input
    assert len(keccak256(b"a" * 300)) == 32
    assert keccak256(b"a" * 136) != keccak256(b"a" * 135)


def test_curve_basics():
    assert bn.g1_is_on_curve(bn.G1_GEN) and bn.g2_is_on_curve(bn.G2_GEN)
    assert bn.g1_mul(bn.G1_GEN, R_MOD) is None
    assert bn.g2_mul(bn.G2_GEN, R_MOD) is None
    assert bn.g1_mul(bn.G1_GEN, 2) == (
        1368015179489954701390400359078579693043519447331113978918064868415326638035,
        9918110051302171585080402603319702774565515993150576347155970296011118125764)


@pytest.mark.parametrize("k", [0, 1, 4, 7])
def test_ntt_roundtrip_and_definition(k):
    rng = random.Random(k)
    n = 1 << k
    a = [rng.randrange(R_MOD) for _ in range(n)]
    A = bn.fft(a)
    w = bn.FR_W[k]
    assert A == [sum(a[j] * pow(w, i * j, R_MOD) for j in range(n)) % R_MOD for i in range(n)]
    assert bn.ifft(A) == a


def test_msm_vs_naive():
    rng = random.Random(3)
    pts = [bn.g1_mul(bn.G1_GEN, rng.randrange(1, R_MOD)) for _ in range(20)]
    sc = [rng.randrange(R_MOD) for _ in range(20)]
    naive = None
    for p, s in zip(pts, sc):
        naive = bn.g1_add(naive, bn.g1_mul(p, s))
    assert bn.msm(pts, sc) == naive


def test_zkey_roundtrip():
    c = synth.synth_circuit(4, 2, 3, seed=9)
    zk = plonk.setup(c, 55)
    data = binfmt.write_zkey(zk)
    zk2 = binfmt.read_zkey(data)
    assert binfmt.write_zkey(zk2) == data
    w = binfmt.read_wtns(binfmt.write_wtns(c["witness"]))
    assert w["witness"] == c["witness"] and w["q"] == R_MOD


def test_synth_is_deterministic_and_satisfied():
    a = synth.synth_circuit(6, 3, 4, seed=5)
    b = synth.synth_circuit(6, 3, 4, seed=5)
    assert a == b
    vals = list(a["witness"]) + [0] * a["nAdditions"]
    nw = len(a["witness"])
    vals[0] = 0
    for k, (x, y, ac, bc) in enumerate(a["additions"]):
        vals[nw + k] = (ac * vals[x] + bc * vals[y]) % R_MOD
    for i, (sa, sb, sc, qm, ql, qr, qo, qc) in enumerate(a["constraints"]):
        va, vb, vc = vals[sa], vals[sb], vals[sc]
        e = (qm * va * vb + ql * va + qr * vb + qo * vc + qc) % R_MOD
        if i < 3:
            e = (e - vals[sa]) % R_MOD      # public input gate: a - PI = 0
        assert e == 0


@pytest.mark.parametrize("name", ["p5", "p8"])
def test_golden_fixtures_regenerate(name):
    with open(os.path.join(GOLD, f"{name}.json")) as f:
        meta = json.load(f)
    c = synth.synth_circuit(meta["power"], meta["n_public"], meta["n_inputs"], seed=meta["seed"])
    zk = plonk.setup(c, meta["tau"])
    with open(os.path.join(GOLD, f"{name}.zkey"), "rb") as f:
        assert f.read() == binfmt.write_zkey(zk)
    for bl in ("zero", "fixed"):
        exp = meta["proofs"][bl]
        b = synth.fixed_blindings() if bl == "fixed" else None
        proof, pub = plonk.prove(zk, c["witness"], b)
        assert plonk.proof_to_bytes(proof).hex() == exp["proof_bin"]
        assert plonk.proof_to_json_obj(proof) == exp["proof"]
        assert [str(x) for x in pub] == exp["publicSignals"]
        assert plonk.verify_with_trapdoor(zk, pub, proof, meta["tau"])


def test_verifier_rejects_tampering():
    with open(os.path.join(GOLD, "p5.json")) as f:
        meta = json.load(f)
    with open(os.path.join(GOLD, "p5.zkey"), "rb") as f:
        zk = binfmt.read_zkey(f.read())
    exp = meta["proofs"]["fixed"]
    proof = plonk.proof_from_bytes(bytes.fromhex(exp["proof_bin"]))
    pub = [int(x) for x in exp["publicSignals"]]
    assert plonk.verify_with_trapdoor(zk, pub, proof, meta["tau"])
    for key in ("eval_a", "eval_zw", "eval_r"):
        bad = dict(proof)
        bad[key] = (bad[key] + 1) % R_MOD
        assert not plonk.verify_with_trapdoor(zk, pub, bad, meta["tau"])
    bad = dict(proof)
    bad["A"] = bn.g1_add(bad["A"], bn.G1_GEN)
    assert not plonk.verify_with_trapdoor(zk, pub, bad, meta["tau"])
    assert not plonk.verify_with_trapdoor(zk, [pub[0] + 1] + pub[1:], proof, meta["tau"])


def test_prover_error_paths():
    c = synth.synth_circuit(5, 3, 4, seed=1)
    zk = plonk.setup(c, 77)
    w = list(c["witness"])
    with pytest.raises(plonk.ProverError, match="Invalid witness length"):
        plonk.prove(zk, w[:-1])
    w[10] += 1
    with pytest.raises(plonk.ProverError, match="T Polynomial is not divisible"):
        plonk.prove(zk, w)
