"""Solidity verifier export (snarkjs `zkey export
solidityverifier`, /root/reference/Makefile:57,62, deployed by
/root/reference/deploy-script.js:4-7): nzcb_vk_to_solidity renders the contract from a
binary verification key, and its verifyProof assembly is executed here by the Yul
interpreter of tests/yul.py (EVM word semantics, EIP-196/197/198 precompiles on the
oracle's curve and pairing code) on the golden proofs and on tampered ones.

Host only (no GPU). Parity with snarkjs's template is unpinned: the reference holds no
generated verifier and snarkjs is not on disk; what is pinned is that the contract
accepts exactly what the library's verifier (nzcb_verify) accepts on these proofs."""
import json
import os
import re
import shutil
import subprocess

import pytest

import nzcb
from tests import yul

GOLD = os.path.join(os.path.dirname(__file__), "golden")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gold(name):
    meta = json.load(open(os.path.join(GOLD, f"{name}.json")))
    zkey = open(os.path.join(GOLD, f"{name}.zkey"), "rb").read()
    return meta, zkey


def _proof_words(proof_bin: bytes) -> bytes:
    """The calldata's proof bytes (nzcb_proof_to_calldata) from the binary proof."""
    hexs = nzcb.proof_to_calldata(proof_bin, b"")
    return bytes.fromhex(hexs.split(",")[0][2:])


@pytest.fixture(scope="module")
def p8():
    meta, zkey = _gold("p8")
    vk = nzcb.vk_from_zkey(zkey)
    return meta, vk, nzcb.vk_to_solidity(vk)


def test_contract_constants_match_the_verification_key(p8):
    meta, vk, sol = p8
    js = nzcb.vk_to_json(vk)
    consts, _ = yul.contract_parts(sol)
    assert consts["N"] == 1 << js["power"] and consts["LOG_N"] == js["power"]
    assert consts["N_PUBLIC"] == js["nPublic"] == meta["n_public"]
    assert consts["W1"] == int(js["w"]) and consts["K1"] == int(js["k1"]) and consts["K2"] == int(js["k2"])
    for name in ("Qm", "Ql", "Qr", "Qo", "Qc", "S1", "S2", "S3"):
        x, y, z = (int(v) for v in js[name])
        assert (consts[f"{name.upper()}_X"], consts[f"{name.upper()}_Y"]) == ((x, y) if z else (0, 0))
    (xr, xi), (yr, yi) = [[int(v) for v in c] for c in js["X_2"][:2]]
    assert (consts["X2_X_RE"], consts["X2_X_IM"], consts["X2_Y_RE"], consts["X2_Y_IM"]) == (xr, xi, yr, yi)
    from oracle import bn254 as bn
    (gxr, gxi), (gyr, gyi) = bn.G2_GEN
    assert (consts["G2_X_RE"], consts["G2_X_IM"], consts["G2_Y_RE"], consts["G2_Y_IM"]) == (gxr, gxi, gyr, gyi)
    assert consts["R"] == bn.R_MOD and consts["Q"] == bn.P_MOD
    assert re.search(r"function verifyProof\(bytes memory proof, uint256\[\] memory pubSignals\) public view "
                     r"returns \(bool\)", sol)
    assert "proof.length != 800 || pubSignals.length != N_PUBLIC" in sol
    assert sol.count("{") == sol.count("}")


@pytest.mark.parametrize("blinding", ["fixed", "zero"])
def test_contract_accepts_golden_proofs(p8, blinding):
    meta, vk, sol = p8
    exp = meta["proofs"][blinding]
    proof = bytes.fromhex(exp["proof_bin"])
    pubs = [int(x) for x in exp["publicSignals"]]
    pub_le = b"".join(x.to_bytes(32, "little") for x in pubs)
    assert nzcb.verify(vk, proof, pub_le)
    ok, calls = yul.run_verify_proof(sol, _proof_words(proof), pubs)
    assert ok
    assert calls[8] == 1 and calls[7] >= 17 and calls[5] == max(1, meta["n_public"]) + 1


def test_contract_rejects_tampered_proofs(p8):
    meta, vk, sol = p8
    exp = meta["proofs"]["fixed"]
    words = _proof_words(bytes.fromhex(exp["proof_bin"]))
    pubs = [int(x) for x in exp["publicSignals"]]
    r = 21888242871839275222246405745257275088548364400416034343698204186575808495617
    # a changed evaluation (eval_r), a changed public signal, a field element out of range,
    # a commitment moved off the curve
    bad_eval = bytearray(words)
    bad_eval[799] ^= 1
    assert not yul.run_verify_proof(sol, bytes(bad_eval), pubs)[0]
    assert not yul.run_verify_proof(sol, words, [pubs[0] ^ 1] + pubs[1:])[0]
    assert not yul.run_verify_proof(sol, words, [pubs[0] + r] + pubs[1:])[0]
    off_curve = bytearray(words)
    off_curve[63] ^= 1   # A.y
    assert not yul.run_verify_proof(sol, bytes(off_curve), pubs)[0]


def test_contract_transcript_variant_and_names(p8):
    """transcript_public = 0 hashes A || B || C only (nzcb_ctx_set_transcript_public):
    the golden proofs (public inputs hashed) then fail; bad contract names are refused."""
    meta, vk, _ = p8
    exp = meta["proofs"]["fixed"]
    sol0 = nzcb.vk_to_solidity(vk, "Verifier", transcript_public=False)
    assert "contract Verifier {" in sol0
    assert not yul.run_verify_proof(sol0, _proof_words(bytes.fromhex(exp["proof_bin"])),
                                    [int(x) for x in exp["publicSignals"]])[0]
    for bad in ("", "9lives", "a b", "x" * 65):
        with pytest.raises(nzcb.NzcbError):
            nzcb.vk_to_solidity(vk, bad)


def test_node_cli_exports(tmp_path):
    """`zkey export verificationkey|solidityverifier|soliditycalldata` through the Node CLI
    (nzcb-circom_amd/js/cli.js), host only."""
    node = shutil.which("node")
    addon = os.path.join(ROOT, "nzcb-circom_amd", "js", "build", "nzcb.node")
    if not node or not os.path.exists(addon):
        pytest.skip("node or the N-API addon is not available")
    cli = os.path.join(ROOT, "nzcb-circom_amd", "js", "cli.js")
    zkey = os.path.join(GOLD, "p8.zkey")
    sol = tmp_path / "Verifier.sol"
    vkj = tmp_path / "verification_key.json"
    subprocess.run([node, cli, "zkey", "export", "verificationkey", zkey, str(vkj)], check=True)
    subprocess.run([node, cli, "zkey", "export", "solidityverifier", zkey, str(sol), "Verifier"], check=True)
    meta, zk = _gold("p8")
    vk = nzcb.vk_from_zkey(zk)
    assert sol.read_text() == nzcb.vk_to_solidity(vk, "Verifier")
    assert json.loads(vkj.read_text()) == nzcb.vk_to_json(vk)
    exp = meta["proofs"]["fixed"]
    (tmp_path / "proof.json").write_text(json.dumps(exp["proof"]))
    (tmp_path / "public.json").write_text(json.dumps(exp["publicSignals"]))
    out = subprocess.run([node, cli, "zkey", "export", "soliditycalldata", str(tmp_path / "public.json"),
                          str(tmp_path / "proof.json")], check=True, capture_output=True, text=True).stdout.strip()
    pub_le = b"".join(int(x).to_bytes(32, "little") for x in exp["publicSignals"])
    assert out == nzcb.proof_to_calldata(bytes.fromhex(exp["proof_bin"]), pub_le)
