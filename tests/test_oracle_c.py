"""The C restatement (oracle/c/nzcb_ref.c) agrees bit-for-bit with the golden
fixtures and with oracle/plonk.py run live; it is the large-size checker and the
CPU baseline (bench.py cpu_baseline, kind "port")."""
import json
import os
import random

import pytest

from oracle import binfmt, bn254 as bn, cbind, plonk, synth
from oracle.bn254 import R_MOD

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("name", ["p5", "p8"])
@pytest.mark.parametrize("bl", ["zero", "fixed"])
def test_c_port_golden(name, bl):
    with open(os.path.join(GOLD, f"{name}.json")) as f:
        meta = json.load(f)
    with open(os.path.join(GOLD, f"{name}.zkey"), "rb") as f:
        z = f.read()
    with open(os.path.join(GOLD, f"{name}.wtns"), "rb") as f:
        w = f.read()
    exp = meta["proofs"][bl]
    b = bytes.fromhex(exp["blinding"]) if exp["blinding"] else None
    proof, pub, _ = cbind.prove(z, w, b, True, 4, 3)
    assert proof.hex() == exp["proof_bin"]
    assert [str(int.from_bytes(pub[i:i + 32], "little")) for i in range(0, 96, 32)] == exp["publicSignals"]


@pytest.mark.parametrize("power,seed,tp", [(10, 31, True), (11, 32, False)])
def test_c_port_vs_python_live(power, seed, tp):
    c = synth.synth_circuit(power, 3, 6, seed=seed)
    zk = plonk.setup(c, 31337 + seed)
    bl = synth.fixed_blindings()
    proof, pub = plonk.prove(zk, c["witness"], bl, transcript_pub=tp)
    got, _, _ = cbind.prove(binfmt.write_zkey(zk), binfmt.write_wtns(c["witness"]),
                            b"".join(x.to_bytes(32, "little") for x in bl), tp, 8, 3)
    assert got == plonk.proof_to_bytes(proof)


def test_c_port_errors():
    with open(os.path.join(GOLD, "p5.zkey"), "rb") as f:
        z = f.read()
    c = synth.synth_circuit(5, 3, 4, seed=1)
    w = list(c["witness"])
    with pytest.raises(RuntimeError, match="Invalid witness length"):
        cbind.prove(z, binfmt.write_wtns(w[:-1]))
    w[7] += 1
    with pytest.raises(RuntimeError, match="T Polynomial is not divisible"):
        cbind.prove(z, binfmt.write_wtns(w))


def test_c_msm_vs_python():
    rng = random.Random(4)
    pts = [bn.g1_mul(bn.G1_GEN, rng.randrange(1, R_MOD)) for _ in range(200)]
    sc = [rng.randrange(R_MOD) for _ in range(200)] + [0, 1, R_MOD - 1]
    pts += [pts[0], pts[1], None]
    got = cbind.msm(b"".join(bn.g1_to_lem(p) for p in pts), b"".join(bn.to_lem(s, R_MOD) for s in sc), 4)
    want = bn.msm(pts, sc)
    assert (bn.from_le(got[:32]), bn.from_le(got[32:])) == want
