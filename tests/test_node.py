"""The Node.js drop-in (nzcb-circom_amd/js: N-API addon + snarkjs-compatible
plonk.prove / plonk.fullProve), driven through `node` as the reference's callers would."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JS = os.path.join(ROOT, "nzcb-circom_amd", "js")
GOLD = os.path.join(ROOT, "tests", "golden")
ADDON = os.path.join(JS, "build", "nzcb.node")

needs_node = pytest.mark.skipif(shutil.which("node") is None or not os.path.exists(ADDON),
                                reason="node or the built addon is unavailable")


def run_node(script: str, timeout=300):
    p = subprocess.run(["node", "-e", script], capture_output=True, text=True, timeout=timeout, cwd=JS)
    assert p.returncode == 0, p.stderr
    return p.stdout


@needs_node
def test_addon_exports():
    out = run_node("const m=require('./'); console.log(JSON.stringify({v: m.version(), "
                   "p: typeof m.plonk.prove, f: typeof m.plonk.fullProve, w: typeof m.wtns.calculate}))")
    d = json.loads(out)
    assert "gfx950" in d["v"] and d["p"] == d["f"] == d["w"] == "function"


@needs_node
def test_program_input_encoding():
    """fullProve's input signals as 32-byte LE field elements (js/index.js putSignal): small
    numbers take a direct path, everything else (numbers past 2^48, strings, BigInts,
    negatives) is reduced mod r, as circom's calculator reduces them; arrays flatten."""
    R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
    vals = [0, 1, 255, (1 << 48) - 1, 1 << 48, (1 << 53) - 1, -1, -7]
    strs = ["12345678901234567890123456789", str(R + 5), str(R - 1)]
    script = ("const m=require('./'); const meta={names:[['a',%d],['b',%d],['c',1]]};"
              "const buf=m._programInputBuffer({a:%s, b:%s, c:BigInt('%d')}, meta);"
              "console.log(buf.toString('hex'))" % (len(vals), len(strs), json.dumps(vals), json.dumps(strs), R + 9))
    got = bytes.fromhex(run_node(script).strip())
    want = b"".join((int(x) % R).to_bytes(32, "little") for x in vals + strs + [R + 9])
    assert got == want


@needs_node
def test_node_zkey_export_past_2gib(tmp_path):
    """zKey.exportVerificationKey / exportSolidityVerifier on a zkey file past
    Node's 2 GiB readFileSync limit (nzcp_live_final.zkey is ~3.9 GB): a golden zkey grown to
    3 GiB by a sparse tail exports the same key and contract as the library's."""
    import nzcb
    big = tmp_path / "big.zkey"
    big.write_bytes(open(os.path.join(GOLD, "p8.zkey"), "rb").read())
    with open(big, "r+b") as f:
        f.truncate(3 << 30)
    script = f"""
const m = require('./');
(async () => {{
  const vk = await m.zKey.exportVerificationKey('{big}');
  const sol = await m.zKey.exportSolidityVerifier('{big}', null, null, {{name: 'Verifier'}});
  console.log(JSON.stringify({{vk, sol}}));
}})().catch((e) => {{ console.error(e); process.exit(1); }});
"""
    d = json.loads(run_node(script))
    vk = nzcb.vk_from_zkey(os.path.join(GOLD, "p8.zkey"))
    assert d["vk"] == nzcb.vk_to_json(vk)
    assert d["sol"] == nzcb.vk_to_solidity(vk, "Verifier")


@needs_node
def test_node_remap_program_matches_library(tmp_path):
    """wtns.remapProgram (nzcb_wprog_remap through N-API) gives the library's bytes; an
    unmatched .sym fails with .unmatched set."""
    import nzcb
    from nzcb import nzcpgen
    from test_wprog_remap import permuted_sym
    c = nzcpgen.wrapper_circuit("readMapLength_test")
    sym, _ = permuted_sym(c, 9)
    for name, data in (("p.nzwp", c.write_program()), ("own.sym", c.write_sym()), ("t.sym", sym),
                       ("bad.sym", sym.replace(b"main.len", b"main.nope"))):
        (tmp_path / name).write_bytes(data)
    script = f"""
const m = require('./');
const fs = require('fs');
const out = m.wtns.remapProgram('{tmp_path}/p.nzwp', '{tmp_path}/own.sym', '{tmp_path}/t.sym');
fs.writeFileSync('{tmp_path}/mapped.nzwp', out);
let bad = null;
try {{ m.wtns.remapProgram('{tmp_path}/p.nzwp', '{tmp_path}/own.sym', '{tmp_path}/bad.sym'); }}
catch (e) {{ bad = {{unmatched: e.unmatched, code: e.code}}; }}
console.log(JSON.stringify({{bad}}));
"""
    d = json.loads(run_node(script))
    assert (tmp_path / "mapped.nzwp").read_bytes() == nzcb.wprog_remap(c.write_program(), c.write_sym(), sym)
    assert d["bad"] == {"unmatched": 1, "code": 2}


@needs_node
@pytest.mark.gpu
def test_node_plonk_prove_golden():
    meta = json.load(open(os.path.join(GOLD, "p8.json")))
    exp = meta["proofs"]["fixed"]
    script = f"""
const m = require('./');
const lines = [];
(async () => {{
  const bl = Buffer.from('{exp['blinding']}', 'hex');
  const r = await m.plonk.prove('{GOLD}/p8.zkey', '{GOLD}/p8.wtns', {{debug: (s) => lines.push(s)}}, {{blinding: bl}});
  // two concurrent proofs on the same (cached) context run on two of its lanes
  const [a, b] = await Promise.all([
    m.plonk.prove('{GOLD}/p8.zkey', '{GOLD}/p8.wtns', null, {{blinding: bl}}),
    m.plonk.prove({{type: 'mem', data: require('fs').readFileSync('{GOLD}/p8.zkey')}}, '{GOLD}/p8.wtns', null, {{blinding: bl}})]);
  console.log(JSON.stringify({{r, a, b, lines}}));
}})().catch((e) => {{ console.error(e); process.exit(1); }});
"""
    d = json.loads(run_node(script))
    for k in ("r", "a", "b"):
        assert d[k]["proof"] == exp["proof"]
        assert d[k]["publicSignals"] == exp["publicSignals"]
    assert "multiexp A" in d["lines"]


@needs_node
@pytest.mark.gpu
def test_node_errors_reject_with_snarkjs_text():
    script = f"""
const m = require('./');
const fs = require('fs');
(async () => {{
  const w = fs.readFileSync('{GOLD}/p8.wtns');
  w[76 + 32 * 20] ^= 1;   // corrupt one witness value
  try {{ await m.plonk.prove('{GOLD}/p8.zkey', w); console.log('no error'); }}
  catch (e) {{ console.log(JSON.stringify({{msg: e.message, code: e.code}})); }}
}})();
"""
    d = json.loads(run_node(script))
    assert d["msg"] == "T Polynomial is not divisible" and d["code"] == 7


@needs_node
@pytest.mark.gpu
def test_cli_plonk_prove_verifies(tmp_path):
    """`node cli.js plonk prove` (the `snarkjs plonk prove` CLI shape): random blinding,
    proof accepted by the oracle's trapdoor verifier."""
    from oracle import binfmt, plonk
    meta = json.load(open(os.path.join(GOLD, "p8.json")))
    pf, pb = tmp_path / "proof.json", tmp_path / "public.json"
    p = subprocess.run(["node", os.path.join(JS, "cli.js"), "plonk", "prove", os.path.join(GOLD, "p8.zkey"),
                        os.path.join(GOLD, "p8.wtns"), str(pf), str(pb)], capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr
    proof = json.loads(pf.read_text())
    pub = [int(x) for x in json.loads(pb.read_text())]
    assert [str(x) for x in pub] == meta["proofs"]["fixed"]["publicSignals"]
    pt = {k: (None if proof[k][2] == "0" else (int(proof[k][0]), int(proof[k][1]))) for k in plonk.PROOF_POINTS}
    pt.update({k: int(proof[k]) for k in plonk.PROOF_EVALS})
    zk = binfmt.read_zkey(open(os.path.join(GOLD, "p8.zkey"), "rb").read())
    assert plonk.verify_with_trapdoor(zk, pub, pt, meta["tau"])


@needs_node
def test_cli_plonk_verify(tmp_path):
    """`node cli.js plonk verify <verification_key.json> <public.json> <proof.json>` (the
    `snarkjs plonk verify` verb): the golden proof prints OK! and exits 0; a
    tampered evaluation or public signal prints "Invalid proof" and exits 1. Host only."""
    meta = json.load(open(os.path.join(GOLD, "p8.json")))
    vk = tmp_path / "verification_key.json"
    p = subprocess.run(["node", os.path.join(JS, "cli.js"), "zkey", "export", "verificationkey",
                        os.path.join(GOLD, "p8.zkey"), str(vk)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    exp = meta["proofs"]["fixed"]

    def verify(proof, pub):
        pf, pb = tmp_path / "proof.json", tmp_path / "public.json"
        pf.write_text(json.dumps(proof))
        pb.write_text(json.dumps(pub))
        return subprocess.run(["node", os.path.join(JS, "cli.js"), "plonk", "verify", str(vk), str(pb), str(pf)],
                              capture_output=True, text=True, timeout=120)

    ok = verify(exp["proof"], exp["publicSignals"])
    assert ok.returncode == 0 and ok.stdout.strip() == "OK!", ok.stderr
    bad_proof = dict(exp["proof"], eval_a=str((int(exp["proof"]["eval_a"]) + 1)))
    r = verify(bad_proof, exp["publicSignals"])
    assert r.returncode == 1 and r.stdout.strip() == "Invalid proof"
    bad_pub = [str(int(exp["publicSignals"][0]) + 1)] + exp["publicSignals"][1:]
    r = verify(exp["proof"], bad_pub)
    assert r.returncode == 1 and r.stdout.strip() == "Invalid proof"


EXAMPLE_PASS_URI = (  # /root/reference/test/nzcp.js:71 (MoH example pass)
    "NZCP:/1/2KCEVIQEIVVWK6JNGEASNICZAEP2KALYDZSGSZB2O5SWEOTOPJRXALTDN53GSZBRHEXGQZLBNR2GQLTOPICRUYMBTIFAIGTUKBAA"
    "UYTWMOSGQQDDN5XHIZLYOSBHQJTIOR2HA4Z2F4XXO53XFZ3TGLTPOJTS6MRQGE4C6Y3SMVSGK3TUNFQWY4ZPOYYXQKTIOR2HA4Z2F4XW46"
    "TDOAXGG33WNFSDCOJONBSWC3DUNAXG46RPMNXW45DFPB2HGL3WGFTXMZLSONUW63TFGEXDALRQMR2HS4DFQJ2FMZLSNFTGSYLCNRSUG4TF"
    "MRSW45DJMFWG6UDVMJWGSY2DN53GSZCQMFZXG4LDOJSWIZLOORUWC3CTOVRGUZLDOSRWSZ3JOZSW4TTBNVSWISTBMNVWUZTBNVUWY6KO"
    "MFWWKZ2TOBQXE4TPO5RWI33CNIYTSNRQFUYDILJRGYDVAYFE6VGU4MCDGK7DHLLYWHVPUS2YIDJOA6Y524TD3AZRM263WTY2BE4DPKIF"
    "27WKF3UDNNVSVWRDYIYVJ65IRJJJ6Z25M2DO4YZLBHWFQGVQR5ZLIWEQJOZTS3IQ7JTNCFDX")


@needs_node
def test_nzcp_input_preparation_kats():
    """pass URI -> ToBeSigned -> circuit input / expected public
    signals, pinned by the reference test's KATs (test/utils.js:16-20 SHA-256 chunks of
    the example ToBeSigned, test/nzcp.js:18,36 nullifier and data) and SURVEY.md §8c."""
    import hashlib
    script = f"""
const z = require('./').nzcp;
const uri = '{EXAMPLE_PASS_URI}';
const data = Buffer.from([...Array(20).keys()].map((i) => i + 1));
const inp = z.circuitInput(uri, data, z.EXAMPLE_TOBESIGNED_MAX);
console.log(JSON.stringify({{tbs: z.toBeSigned(uri).toString('hex'), claims: z.claims(uri),
  pub: z.expectedPublicSignals(uri, data), inp}}));
"""
    d = json.loads(run_node(script))
    tbs = bytes.fromhex(d["tbs"])
    assert len(tbs) == 314
    # reference KAT: sha256(ToBeSigned) as two LSB-first chunks of 248 bits (test/utils.js:11-19)
    chunks = [366677313775235426412199931337625106565467678080892143469223808086055532772, 119]
    bits = [(c >> j) & 1 for c in chunks for j in range(248)]
    kat = bytes(sum(bits[8 * i + t] << (7 - t) for t in range(8)) for i in range(32))
    assert hashlib.sha256(tbs).digest() == kat
    assert d["claims"]["exp"] == 1951416330
    assert f"{d['claims']['givenName']},{d['claims']['familyName']},{d['claims']['dob']}" == "Jack,Sparrow,1960-04-16"
    assert d["pub"] == [
        "8464235439336389695359576364537904521787463454426143836621154307990710930",
        "334204042160295982690797293769892102755483197293558786265320143920457223185",
        "430989588176824417852954207888075491695208395262355815151652761069951123456"]
    inp = d["inp"]
    assert inp["toBeSignedLen"] == 314 and len(inp["toBeSigned"]) == 314 * 8 and len(inp["data"]) == 160
    assert bytes(sum(inp["toBeSigned"][8 * i + t] << (7 - t) for t in range(8)) for i in range(314)) == tbs
    # data: bytes reversed, bits reversed within each byte (EVM rearrangement)
    dbytes = bytes(sum(inp["data"][8 * i + t] << (7 - t) for t in range(8)) for i in range(20))
    assert dbytes == bytes(int(f"{b:08b}"[::-1], 2) for b in reversed(range(1, 21)))


@needs_node
@pytest.mark.gpu
def test_node_nzcp_witness_on_gpu():
    """Node nzcp.witness (addon.nzcpWitness -> nzcb_nzcp_witness): the example pass in the
    example circuit gives the reference test's public signals; a pass in
    the wrong circuit throws like calculateWitness."""
    script = f"""
const n = require('./');
const z = n.nzcp;
const uri = '{EXAMPLE_PASS_URI}';
const data = Buffer.from([...Array(20).keys()].map((i) => i + 1));
const r = z.witness(z.circuitInput(uri, data, z.EXAMPLE_TOBESIGNED_MAX), {{circuit: 'example'}});
let threw = '';
try {{ z.witness(z.circuitInput(uri, data, z.LIVE_TOBESIGNED_MAX)); }} catch (e) {{ threw = e.message; }}
console.log(JSON.stringify({{r, expected: z.expectedPublicSignals(uri, data), threw}}));
"""
    d = json.loads(run_node(script))
    assert d["r"]["publicSignals"] == d["expected"]
    assert d["r"]["vcPos"] == 76 and d["r"]["nullifier"] == "Jack,Sparrow,1960-04-16"
    assert d["r"]["toBeSignedHash"] == "271ce33d671a2d3b816d788135f4343e14bc66802f8cd841faac939e8c11f3ee"
    assert "CBOR type is not a map" in d["threw"]


@needs_node
@pytest.mark.gpu
def test_cli_plonk_setup_matches_library(tmp_path):
    """`node cli.js plonk setup <r1cs> <ptau> <zkey>` (/root/reference/Makefile:55,60) writes
    the zkey nzcb_plonk_setup builds, which tests/test_r1cs_setup.py checks against the
    oracle and proves with."""
    import nzcb
    from oracle import r1cs
    data, _ = r1cs.random_r1cs(31, n_steps=30)
    ptau = r1cs.write_ptau(0x5E7A9, 8)
    (tmp_path / "c.r1cs").write_bytes(data)
    (tmp_path / "p.ptau").write_bytes(ptau)
    zf = tmp_path / "c.zkey"
    p = subprocess.run(["node", os.path.join(JS, "cli.js"), "plonk", "setup", str(tmp_path / "c.r1cs"),
                        str(tmp_path / "p.ptau"), str(zf)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    assert zf.read_bytes() == nzcb.plonk_setup(data, ptau)


@needs_node
@pytest.mark.gpu
def test_node_full_prove_wasm_and_witness_program(tmp_path):
    """plonk.fullProve end to end (configs[0]'s plumbing): a circom-2.0.x-ABI witness .wasm
    (tests/wasm_tiny.py, `c <== a * b`) on the host, and the same circuit's witness program
    on the GPU, give the same witness, hence the same proof under the same blinding; the
    proof verifies and publicSignals = ["33"]. Parity with circom/snarkjs: unpinned."""
    import nzcb
    import wasm_tiny
    r1cs, prog = wasm_tiny.mul_circuit()
    zkey = nzcb.plonk_setup(r1cs, nzcb.ptau_synth(4, 0x1234567))
    (tmp_path / "mul.zkey").write_bytes(zkey)
    (tmp_path / "mul.wasm").write_bytes(wasm_tiny.build_mul_wasm())
    (tmp_path / "mul.wprog").write_bytes(prog)
    bl = b"".join((7 * i + 3 + (i << 200)).to_bytes(32, "little") for i in range(11)).hex()  # fixed, < r
    script = f"""
const m = require('./');
(async () => {{
  const bl = Buffer.from('{bl}', 'hex');
  const z = '{tmp_path}/mul.zkey';
  const a = await m.plonk.fullProve({{a: 3, b: 11}}, '{tmp_path}/mul.wasm', z, null, {{blinding: bl}});
  const g = await m.plonk.fullProve({{b: 11, a: 3}}, '{tmp_path}/mul.wprog', z, null, {{blinding: bl}});
  const vk = await m.zKey.exportVerificationKey(z);
  const ok = await m.plonk.verify(vk, g.publicSignals, g.proof);
  let err = '';
  try {{ await m.plonk.fullProve({{a: 3}}, '{tmp_path}/mul.wprog', z); }} catch (e) {{ err = e.message; }}
  console.log(JSON.stringify({{a, g, ok, err}}));
}})().catch((e) => {{ console.error(e); process.exit(1); }});
"""
    d = json.loads(run_node(script))
    assert d["a"]["publicSignals"] == ["33"] == d["g"]["publicSignals"]
    assert d["a"]["proof"] == d["g"]["proof"]
    assert d["ok"] is True
    assert d["err"].startswith("Signal b not found")


@needs_node
@pytest.mark.gpu
def test_node_concurrent_full_prove_matches_sequential(tmp_path):
    """concurrent plonk.fullProve promises on one context feed its lanes
    (nzcb_prove_logged per call, no per-context lock) and keep the witness in HBM
    (fullProveDevice). 8 concurrent calls with fixed blinding, over 3 lanes (so calls wait
    for a lane), give the same proofs as the same 8 calls made one after another; each call's
    logger sees only its own proof's lines."""
    import nzcb
    import wasm_tiny
    r1cs, prog = wasm_tiny.mul_circuit()
    zkey = nzcb.plonk_setup(r1cs, nzcb.ptau_synth(4, 0x1234567))
    (tmp_path / "mul.zkey").write_bytes(zkey)
    (tmp_path / "mul.wprog").write_bytes(prog)
    bl = b"".join((7 * i + 3 + (i << 200)).to_bytes(32, "little") for i in range(11)).hex()
    script = f"""
const m = require('./');
(async () => {{
  const bl = Buffer.from('{bl}', 'hex');
  const z = '{tmp_path}/mul.zkey', p = '{tmp_path}/mul.wprog';
  const opts = {{blinding: bl, lanes: 3}};
  const seq = [];
  for (let a = 2; a < 10; a++) seq.push(await m.plonk.fullProve({{a, b: 11}}, p, z, null, opts));
  const logs = [];
  const con = await Promise.all([...Array(8).keys()].map((i) => {{
    const lines = [];
    logs.push(lines);
    return m.plonk.fullProve({{a: i + 2, b: 11}}, p, z, {{debug: (s) => lines.push(s)}}, opts);
  }}));
  const vk = await m.zKey.exportVerificationKey(z);
  const ok = await Promise.all(con.map((r) => m.plonk.verify(vk, r.publicSignals, r.proof)));
  console.log(JSON.stringify({{seq, con, ok, logs: logs.map((l) => l.filter((x) => x === 'multiexp A').length)}}));
}})().catch((e) => {{ console.error(e); process.exit(1); }});
"""
    d = json.loads(run_node(script))
    assert d["seq"] == d["con"]
    assert [r["publicSignals"] for r in d["con"]] == [[str(11 * a)] for a in range(2, 10)]
    assert all(d["ok"])
    assert d["logs"] == [1] * 8


@needs_node
@pytest.mark.gpu
def test_node_reused_buffer_is_rehashed(tmp_path):
    """contexts and witness programs are cached by Buffer identity; a Buffer whose
    contents are replaced by another zkey of the same length (same circuit, other tau) must
    not reuse the old context: each proof verifies under its own key and not the other."""
    import nzcb
    import wasm_tiny
    r1cs, prog = wasm_tiny.mul_circuit()
    z1 = nzcb.plonk_setup(r1cs, nzcb.ptau_synth(4, 0x1234567))
    z2 = nzcb.plonk_setup(r1cs, nzcb.ptau_synth(4, 0x7654321))
    assert len(z1) == len(z2) and z1 != z2
    (tmp_path / "z1.zkey").write_bytes(z1)
    (tmp_path / "z2.zkey").write_bytes(z2)
    (tmp_path / "mul.wprog").write_bytes(prog)
    script = f"""
const m = require('./');
const fs = require('fs');
(async () => {{
  const buf = Buffer.from(fs.readFileSync('{tmp_path}/z1.zkey'));
  const p = fs.readFileSync('{tmp_path}/mul.wprog');
  const r1 = await m.plonk.fullProve({{a: 3, b: 11}}, p, buf);
  fs.readFileSync('{tmp_path}/z2.zkey').copy(buf);          // same Buffer, other zkey
  const r2 = await m.plonk.fullProve({{a: 3, b: 11}}, p, buf);
  const vk1 = await m.zKey.exportVerificationKey('{tmp_path}/z1.zkey');
  const vk2 = await m.zKey.exportVerificationKey('{tmp_path}/z2.zkey');
  console.log(JSON.stringify({{
    v11: await m.plonk.verify(vk1, r1.publicSignals, r1.proof), v22: await m.plonk.verify(vk2, r2.publicSignals, r2.proof),
    v12: await m.plonk.verify(vk1, r2.publicSignals, r2.proof)}}));
}})().catch((e) => {{ console.error(e); process.exit(1); }});
"""
    d = json.loads(run_node(script))
    assert d == {"v11": True, "v22": True, "v12": False}


@needs_node
@pytest.mark.gpu
def test_node_full_prove_on_second_device(tmp_path):
    """fullProve with {device: 1} keeps the witness program, its HBM buffers and the
    context on device 1 (the per-call thread allocates on the program's device). Skipped
    on a one-GPU box."""
    import nzcb
    import wasm_tiny
    if nzcb.device_count() < 2:
        pytest.skip("one GPU")
    r1cs, prog = wasm_tiny.mul_circuit()
    (tmp_path / "mul.zkey").write_bytes(nzcb.plonk_setup(r1cs, nzcb.ptau_synth(4, 0x1234567)))
    (tmp_path / "mul.wprog").write_bytes(prog)
    bl = b"".join((7 * i + 3 + (i << 200)).to_bytes(32, "little") for i in range(11)).hex()
    script = f"""
const m = require('./');
(async () => {{
  const bl = Buffer.from('{bl}', 'hex');
  const z = '{tmp_path}/mul.zkey', p = '{tmp_path}/mul.wprog';
  const d0 = await m.plonk.fullProve({{a: 3, b: 11}}, p, z, null, {{blinding: bl}});
  const d1 = await m.plonk.fullProve({{a: 3, b: 11}}, p, z, null, {{blinding: bl, device: 1}});
  console.log(JSON.stringify({{d0, d1}}));
}})().catch((e) => {{ console.error(e); process.exit(1); }});
"""
    d = json.loads(run_node(script))
    assert d["d0"] == d["d1"] and d["d1"]["publicSignals"] == ["33"]


@needs_node
@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_node_full_prove_nzcp_live(tmp_path):
    """plonk.fullProve of the real nzcp_live circuit from Node: the test/nzcp.js-shaped input
    object, the GPU witness program, a 3.9 GB zkey read by file name (memory-mapped by the
    library). publicSignals equal the CPU restatement's outputs; the proof verifies."""
    import ctypes
    import nzcb
    import nzcp_cases as C
    from nzcb import nzcp, nzcplive
    from oracle import nzcp_circuit as nz
    r1cs, prog, _ = nzcplive.build()
    zp, zl = nzcplive.setup_raw(r1cs)
    try:
        with open(tmp_path / "live.zkey", "wb") as f:
            f.write((ctypes.c_uint8 * zl).from_address(zp))
        vk = nzcb.vk_to_json(nzcb.vk_from_zkey((zp, zl)))
    finally:
        nzcb.free_ptr(zp)
    (tmp_path / "live.wprog").write_bytes(prog)
    (tmp_path / "vk.json").write_text(json.dumps(vk))
    tbs = nzcp.pass_tbs(live=True)
    inp = nzcp.circuit_input(tbs, bytes(range(1, 21)))
    (tmp_path / "input.json").write_text(json.dumps(inp))
    want = C.oracle_record(C.case("live", nz.LIVE_PARAMS, tbs, data=bytes(range(1, 21))))["out"]
    script = f"""
const m = require('./');
const fs = require('fs');
(async () => {{
  const input = JSON.parse(fs.readFileSync('{tmp_path}/input.json'));
  const r = await m.plonk.fullProve(input, '{tmp_path}/live.wprog', '{tmp_path}/live.zkey');
  const vk = JSON.parse(fs.readFileSync('{tmp_path}/vk.json'));
  const ok = await m.plonk.verify(vk, r.publicSignals, r.proof);
  console.log(JSON.stringify({{pub: r.publicSignals, ok}}));
}})().catch((e) => {{ console.error(e); process.exit(1); }});
"""
    d = json.loads(run_node(script, timeout=600))
    assert d["pub"] == [str(v) for v in want]
    assert d["ok"] is True


@needs_node
@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_node_full_prove_nzcp_example_moh_pass(tmp_path):
    """configs[0]: plonk.fullProve of nzcp_example (NZCPPubIdentity(0,314,0,4,2,4),
    /root/reference/circuits/nzcp_example.circom) on the Ministry of Health example pass
    (test/nzcp.js:71), input built as test/nzcp.js:33-42 does, from Node. publicSignals are
    SURVEY.md §8c's three values (pinned by the reference's decode at test/nzcp.js:44-68);
    the proof verifies."""
    import ctypes
    import nzcb
    from nzcb import nzcp, nzcpgen, nzcplive
    r1cs, prog, _ = nzcplive.build(nzcpgen.EXAMPLE)
    zp, zl = nzcplive.setup_raw(r1cs)
    try:
        with open(tmp_path / "example.zkey", "wb") as f:
            f.write((ctypes.c_uint8 * zl).from_address(zp))
        vk = nzcb.vk_to_json(nzcb.vk_from_zkey((zp, zl)))
    finally:
        nzcb.free_ptr(zp)
    (tmp_path / "example.wprog").write_bytes(prog)
    (tmp_path / "vk.json").write_text(json.dumps(vk))
    tbs = nzcp.to_be_signed(nzcp.EXAMPLE_PASS_URI)
    inp = nzcp.circuit_input(tbs, bytes(range(1, 21)), nzcp.EXAMPLE_TOBESIGNED_MAX)
    (tmp_path / "input.json").write_text(json.dumps(inp))
    script = f"""
const m = require('./');
const fs = require('fs');
(async () => {{
  const input = JSON.parse(fs.readFileSync('{tmp_path}/input.json'));
  const r = await m.plonk.fullProve(input, '{tmp_path}/example.wprog', '{tmp_path}/example.zkey');
  const vk = JSON.parse(fs.readFileSync('{tmp_path}/vk.json'));
  const ok = await m.plonk.verify(vk, r.publicSignals, r.proof);
  console.log(JSON.stringify({{pub: r.publicSignals, ok}}));
}})().catch((e) => {{ console.error(e); process.exit(1); }});
"""
    d = json.loads(run_node(script, timeout=600))
    assert d["pub"] == ["8464235439336389695359576364537904521787463454426143836621154307990710930",
                        "334204042160295982690797293769892102755483197293558786265320143920457223185",
                        "430989588176824417852954207888075491695208395262355815151652761069951123456"]
    assert d["ok"] is True
