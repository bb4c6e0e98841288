"""Verification key export, pairing verifier and Solidity calldata (SURVEY.md §8f
ranks 1 and 4): the host C-ABI (nzcb_vk_from_zkey / nzcb_verify / nzcb_proof_to_calldata,
no GPU needed) against the CPU oracle, whose pairing is pinned by bilinearity and by the
trapdoor check tau * lhs == rhs of the synthetic setup. Parity with snarkjs unpinned
(no snarkjs vk / calldata fixtures exist offline)."""
import json
import os
import shutil
import subprocess

import pytest

import nzcb
from oracle import binfmt, bn254 as bn, pairing, plonk, synth

GOLD = os.path.join(os.path.dirname(__file__), "golden")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gold(name):
    meta = json.load(open(os.path.join(GOLD, f"{name}.json")))
    zkey = open(os.path.join(GOLD, f"{name}.zkey"), "rb").read()
    return meta, zkey


def _pub_bytes(pub):
    return b"".join(int(x).to_bytes(32, "little") for x in pub)


def test_pairing_bilinear_nondegenerate():
    P, Q = bn.G1_GEN, bn.G2_GEN
    e = pairing.pairing(Q, P)
    assert e != pairing.f12_one()
    assert pairing.f12_pow(e, bn.R_MOD) == pairing.f12_one()
    a, b = 12345, 67890
    assert pairing.pairing(bn.g2_mul(Q, b), bn.g1_mul(P, a)) == pairing.f12_pow(e, a * b)
    assert pairing.pairing_check([(bn.g1_mul(P, a), bn.g2_mul(Q, b)), (bn.g1_neg(bn.g1_mul(P, a * b)), Q)])
    assert not pairing.pairing_check([(bn.g1_mul(P, a), bn.g2_mul(Q, b)), (bn.g1_neg(P), Q)])


@pytest.mark.parametrize("name", ["p5", "p8"])
def test_vk_json_matches_oracle(name):
    meta, zkey = _gold(name)
    vk = nzcb.vk_from_zkey(zkey)
    got = nzcb.vk_to_json(vk)
    want = json.loads(json.dumps(plonk.vk_to_json_obj(plonk.vk_from_zkey(binfmt.read_zkey(zkey)))))
    assert got == want
    assert list(got.keys()) == ["protocol", "curve", "nPublic", "power", "k1", "k2", "Qm", "Ql", "Qr", "Qo",
                                "Qc", "S1", "S2", "S3", "X_2", "w"]
    assert nzcb.vk_from_json(got) == vk


def test_vk_from_zkey_file_past_2gib(tmp_path):
    """`zkey export` on nzcp_live's ~3.9 GB zkey. The path entry
    (nzcb_vk_from_zkey_file) maps the file: a golden zkey grown to 3 GiB by a sparse tail
    (the reader ignores bytes past the sections) gives the same key; a missing file fails."""
    meta, zkey = _gold("p8")
    big = tmp_path / "big.zkey"
    big.write_bytes(zkey)
    with open(big, "r+b") as f:
        f.truncate(3 << 30)
    assert os.path.getsize(big) > (2 << 30)
    assert nzcb.vk_from_zkey(str(big)) == nzcb.vk_from_zkey(zkey)
    with pytest.raises(nzcb.NzcbError, match="cannot open"):
        nzcb.vk_from_zkey(str(tmp_path / "missing.zkey"))


@pytest.mark.parametrize("name", ["p5", "p8"])
@pytest.mark.parametrize("bl", ["zero", "fixed"])
def test_verify_golden_and_tampered(name, bl):
    meta, zkey = _gold(name)
    exp = meta["proofs"][bl]
    vk = nzcb.vk_from_zkey(zkey)
    proof = bytes.fromhex(exp["proof_bin"])
    pub = _pub_bytes(exp["publicSignals"])
    zk = binfmt.read_zkey(zkey)
    ovk = plonk.vk_from_zkey(zk)
    op = plonk.proof_from_bytes(proof)
    opub = [int(x) for x in exp["publicSignals"]]
    assert nzcb.verify(vk, proof, pub)
    assert plonk.verify(ovk, opub, op)
    assert plonk.verify_with_trapdoor(zk, opub, op, meta["tau"])
    # every evaluation, one point and one public signal perturbed: all rejected by both
    cases = []
    for k in plonk.PROOF_EVALS:
        q = dict(op)
        q[k] = (q[k] + 1) % bn.R_MOD
        cases.append((q, opub))
    q = dict(op)
    q["T2"] = bn.g1_add(q["T2"], bn.G1_GEN)
    cases.append((q, opub))
    cases.append((op, [(opub[0] + 1) % bn.R_MOD] + opub[1:]))
    for q, pb in cases:
        assert not nzcb.verify(vk, plonk.proof_to_bytes(q), _pub_bytes(pb))
    assert not plonk.verify(ovk, cases[0][1], cases[0][0])


def test_verify_rejects_malformed():
    meta, zkey = _gold("p5")
    exp = meta["proofs"]["fixed"]
    vk = nzcb.vk_from_zkey(zkey)
    proof = bytearray(bytes.fromhex(exp["proof_bin"]))
    pub = _pub_bytes(exp["publicSignals"])
    off_curve = bytearray(proof)
    off_curve[64] ^= 1  # B.x
    assert not nzcb.verify(vk, bytes(off_curve), pub)
    big = bytearray(proof)
    big[576:608] = (bn.R_MOD + 1).to_bytes(32, "little")  # eval_a >= r
    assert not nzcb.verify(vk, bytes(big), pub)
    assert not nzcb.verify(vk, bytes(proof), pub[:-32])  # wrong number of public signals


def test_verify_transcript_without_public_inputs():
    c = synth.synth_circuit(5, 2, 3, seed=31)
    zk = plonk.setup(c, 777)
    bls = synth.fixed_blindings()
    proof, pub = plonk.prove(zk, c["witness"], bls, transcript_pub=False)
    vk = nzcb.vk_from_zkey(binfmt.write_zkey(zk))
    pb = plonk.proof_to_bytes(proof)
    assert nzcb.verify(vk, pb, _pub_bytes(pub), transcript_public=False)
    assert not nzcb.verify(vk, pb, _pub_bytes(pub), transcript_public=True)
    assert plonk.verify(plonk.vk_from_zkey(zk), pub, proof, transcript_pub=False)


@pytest.mark.parametrize("name", ["p5", "p8"])
def test_calldata_and_json_api(name):
    meta, zkey = _gold(name)
    exp = meta["proofs"]["fixed"]
    proof = bytes.fromhex(exp["proof_bin"])
    opub = [int(x) for x in exp["publicSignals"]]
    cd = nzcb.proof_to_calldata(proof, _pub_bytes(opub))
    assert cd == plonk.solidity_calldata(plonk.proof_from_bytes(proof), opub)
    assert cd.startswith("0x") and len(cd.split(",")[0]) == 2 + 2 * (9 * 64 + 7 * 32)
    vkj = nzcb.vk_to_json(nzcb.vk_from_zkey(zkey))
    assert nzcb.plonk.verify(vkj, exp["publicSignals"], exp["proof"])
    assert nzcb.proof_from_json(exp["proof"]) == proof


@pytest.mark.skipif(shutil.which("node") is None or
                    not os.path.exists(os.path.join(ROOT, "nzcb-circom_amd", "js", "build", "nzcb.node")),
                    reason="node or the built addon is unavailable")
def test_node_verify_vk_calldata():
    meta, _ = _gold("p8")
    exp = meta["proofs"]["fixed"]
    script = f"""
const m = require('./');
(async () => {{
  const vk = await m.zKey.exportVerificationKey('{GOLD}/p8.zkey');
  const e = {json.dumps(exp)};
  const bad = JSON.parse(JSON.stringify(e.proof)); bad.eval_a = (BigInt(bad.eval_a) + BigInt(1)).toString();
  console.log(JSON.stringify({{vk, ok: await m.plonk.verify(vk, e.publicSignals, e.proof),
    bad: await m.plonk.verify(vk, e.publicSignals, bad),
    cd: await m.plonk.exportSolidityCallData(e.proof, e.publicSignals)}}));
}})().catch((err) => {{ console.error(err); process.exit(1); }});
"""
    p = subprocess.run(["node", "-e", script], capture_output=True, text=True, timeout=120,
                       cwd=os.path.join(ROOT, "nzcb-circom_amd", "js"))
    assert p.returncode == 0, p.stderr
    d = json.loads(p.stdout)
    assert d["ok"] is True and d["bad"] is False
    _, zkey = _gold("p8")
    assert d["vk"] == nzcb.vk_to_json(nzcb.vk_from_zkey(zkey))
    assert d["cd"] == nzcb.proof_to_calldata(bytes.fromhex(exp["proof_bin"]), _pub_bytes(exp["publicSignals"]))
