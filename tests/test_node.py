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
  // two concurrent proofs on the same (cached) context are serialized by the library
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
