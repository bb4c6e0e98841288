"""GPU PLONK prover parity through the C-ABI (nzcb_ctx_create / nzcb_prove).

Bit-exact against (a) the committed golden fixtures made by the CPU oracle and
(b) the oracle run live on fresh seeded circuits. Error paths reproduce
snarkjs 0.4.12's exception text.
"""
import json
import os
import struct

import pytest

import nzcb
from oracle import binfmt, plonk, synth

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _gold(name):
    with open(os.path.join(GOLD, f"{name}.json")) as f:
        meta = json.load(f)
    with open(os.path.join(GOLD, f"{name}.zkey"), "rb") as f:
        zkey = f.read()
    with open(os.path.join(GOLD, f"{name}.wtns"), "rb") as f:
        wtns = f.read()
    return meta, zkey, wtns


@pytest.mark.parametrize("name", ["p5", "p8"])
@pytest.mark.parametrize("bl", ["zero", "fixed"])
def test_golden_proof_bits(name, bl):
    meta, zkey, wtns = _gold(name)
    exp = meta["proofs"][bl]
    ctx = nzcb.ProverContext(zkey)
    blinding = bytes.fromhex(exp["blinding"]) if exp["blinding"] else bytes(352)  # explicit zero blinding
    proof, pub = ctx.prove_raw(wtns, blinding)
    assert proof.hex() == exp["proof_bin"]
    res = ctx.prove(wtns, blinding)
    assert res["proof"] == exp["proof"]
    assert res["publicSignals"] == exp["publicSignals"]
    # keys in snarkjs order
    assert list(res["proof"].keys()) == list(exp["proof"].keys())
    ctx.close()


def test_repeat_proofs_same_context():
    meta, zkey, wtns = _gold("p8")
    exp = meta["proofs"]["fixed"]
    ctx = nzcb.ProverContext(zkey)
    bl = bytes.fromhex(exp["blinding"])
    for _ in range(3):
        proof, _ = ctx.prove_raw(wtns, bl)
        assert proof.hex() == exp["proof_bin"]


def test_concurrent_calls_on_lanes_bit_exact():
    """Host threads proving on one context at the same time (the lane pool of
    nzcb_prove_logged: each call takes a free lane, a fifth waits): every proof equals the
    golden one, with the golden blinding and with a per-thread one against sequential
    proofs; the lane count set again unchanged returns at once, as a Node caller does."""
    import threading
    meta, zkey, wtns = _gold("p8")
    exp = meta["proofs"]["fixed"]
    bl = bytes.fromhex(exp["blinding"])
    ctx = nzcb.ProverContext(zkey)
    try:
        ctx.set_lanes(4)
        others = [bytes([(k * 37 + i) % 251 for i in range(352)]) for k in range(5)]
        want = [ctx.prove_raw(wtns, b)[0] for b in others]       # sequential
        res, errs = {}, []

        def worker(k):
            try:
                ctx.set_lanes(4)                                     # no change: returns at once
                res[("gold", k)] = ctx.prove_raw(wtns, bl)[0]
                res[("other", k)] = ctx.prove_raw(wtns, others[k])[0]
            except Exception as e:  # noqa: BLE001 (reported below)
                errs.append(e)
        threads = [threading.Thread(target=worker, args=(k,)) for k in range(5)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(120)
        assert not errs, errs
        assert all(res[("gold", k)].hex() == exp["proof_bin"] for k in range(5))
        assert [res[("other", k)] for k in range(5)] == want
    finally:
        ctx.close()


@pytest.mark.parametrize("power,seed,npub,nin", [(4, 11, 1, 2), (6, 12, 3, 5), (10, 13, 3, 8), (11, 14, 5, 16),
                                                 (7, 16, 8, 10), (7, 17, 10, 12)])
def test_live_oracle(power, seed, npub, nin):
    c = synth.synth_circuit(power, npub, nin, seed=seed)
    tau = 1000003 + seed
    zk = plonk.setup(c, tau)
    zkey = binfmt.write_zkey(zk)
    wtns = binfmt.write_wtns(c["witness"])
    bl = [(seed * 7919 + i * 104729) % plonk.R_MOD if hasattr(plonk, "R_MOD") else 0 for i in range(11)]
    from oracle.bn254 import R_MOD
    bl = [(seed * 7919 + i * 104729 + (i << 200)) % R_MOD for i in range(11)]
    proof, pub = plonk.prove(zk, c["witness"], bl)
    ctx = nzcb.ProverContext(zkey)
    got, gpub = ctx.prove_raw(wtns, b"".join(x.to_bytes(32, "little") for x in bl))
    assert got == plonk.proof_to_bytes(proof)
    assert gpub == b"".join(x.to_bytes(32, "little") for x in pub)
    assert plonk.verify_with_trapdoor(zk, pub, plonk.proof_from_bytes(got), tau)


def test_transcript_without_public_inputs():
    c = synth.synth_circuit(7, 3, 4, seed=21)
    zk = plonk.setup(c, 4242)
    proof, pub = plonk.prove(zk, c["witness"], synth.fixed_blindings(), transcript_pub=False)
    ctx = nzcb.ProverContext(binfmt.write_zkey(zk), transcript_public=False)
    got, _ = ctx.prove_raw(binfmt.write_wtns(c["witness"]),
                           b"".join(x.to_bytes(32, "little") for x in synth.fixed_blindings()))
    assert got == plonk.proof_to_bytes(proof)


def test_logger_lines():
    meta, zkey, wtns = _gold("p5")
    lines = []
    ctx = nzcb.ProverContext(zkey, logger=lines.append)
    ctx.prove_raw(wtns)
    assert "multiexp A" in lines and any(x.startswith("beta: ") for x in lines)


def test_error_witness_length():
    meta, zkey, wtns = _gold("p5")
    w = binfmt.read_wtns(wtns)["witness"][:-1]
    ctx = nzcb.ProverContext(zkey)
    with pytest.raises(nzcb.NzcbError) as ei:
        ctx.prove_raw(binfmt.write_wtns(w))
    assert ei.value.name == "WITNESS_LEN"
    assert str(ei.value).startswith("Invalid witness length. Circuit: ")


def test_error_bad_witness_not_divisible():
    meta, zkey, wtns = _gold("p8")
    w = binfmt.read_wtns(wtns)["witness"]
    w[20] = (w[20] + 1)
    ctx = nzcb.ProverContext(zkey)
    with pytest.raises(nzcb.NzcbError) as ei:
        ctx.prove_raw(binfmt.write_wtns(w))
    assert str(ei.value) == "T Polynomial is not divisible"


def test_error_copy_constraints():
    meta, zkey, wtns = _gold("p8")
    zk = binfmt.read_zkey(zkey)
    # rewire one A-wire of a gate to a different signal: the permutation no longer matches
    zk["aMap"][40] = zk["aMap"][41] if zk["aMap"][41] != zk["aMap"][40] else 1
    ctx = nzcb.ProverContext(binfmt.write_zkey(zk))
    with pytest.raises(nzcb.NzcbError) as ei:
        ctx.prove_raw(wtns)
    assert str(ei.value) == "Copy constraints does not match"


def test_error_not_plonk_and_curve():
    meta, zkey, wtns = _gold("p5")
    bad = bytearray(zkey)
    # section 1 payload (protocol id) starts after the file header (12) + section header (12)
    struct.pack_into("<I", bad, 24, 1)
    with pytest.raises(nzcb.NzcbError) as ei:
        nzcb.ProverContext(bytes(bad))
    assert str(ei.value) == "zkey file is not plonk"
    ctx = nzcb.ProverContext(zkey)
    w = bytearray(wtns)
    # wtns section 1: n8 at offset 24, q at 28..60
    w[28] ^= 1
    with pytest.raises(nzcb.NzcbError) as ei:
        ctx.prove_raw(bytes(w))
    assert str(ei.value) == "Curve of the witness does not match the curve of the proving key"


def test_plonk_prove_api_random_blinding_verifies(tmp_path):
    meta, zkey, wtns = _gold("p8")
    zp = tmp_path / "c.zkey"
    wp = tmp_path / "c.wtns"
    zp.write_bytes(zkey)
    wp.write_bytes(wtns)
    res = nzcb.plonk.prove(str(zp), str(wp))
    proof = res["proof"]
    zk = binfmt.read_zkey(zkey)
    p = {}
    for k in plonk.PROOF_POINTS:
        v = proof[k]
        p[k] = None if v[2] == "0" else (int(v[0]), int(v[1]))
    for k in plonk.PROOF_EVALS:
        p[k] = int(proof[k])
    pub = [int(x) for x in res["publicSignals"]]
    assert plonk.verify_with_trapdoor(zk, pub, p, meta["tau"])


def test_batch_lanes_bit_exact():
    """nzcb_prove_batch over 3 lanes sharing one resident proving key: every proof
    equals its golden fixture, whatever lane ran it (host and device witnesses)."""
    meta, zkey, wtns = _gold("p8")
    w = binfmt.read_wtns(wtns)["witness"]
    wit = b"".join(x.to_bytes(32, "little") for x in w)
    ctx = nzcb.ProverContext(zkey)
    ctx.set_lanes(3)
    assert ctx.lanes == 3
    kinds = ["fixed", "zero", "fixed", "fixed", "zero", "zero", "fixed"]
    bls = [bytes.fromhex(meta["proofs"][k]["blinding"]) if meta["proofs"][k]["blinding"] else bytes(352) for k in kinds]
    res = ctx.prove_batch_raw([wit] * len(kinds), blindings=bls)
    for k, (proof, pub) in zip(kinds, res):
        assert proof.hex() == meta["proofs"][k]["proof_bin"]
    dev = nzcb.dev_alloc(len(wit))
    try:
        nzcb.h2d(dev, wit)
        res = ctx.prove_batch_raw([dev] * 4, n_witness=len(w), blindings=bls[:4], on_device=True)
        for k, (proof, pub) in zip(kinds[:4], res):
            assert proof.hex() == meta["proofs"][k]["proof_bin"]
    finally:
        nzcb.dev_free(dev)
    # single-proof calls still work after the batch (lane 0)
    proof, _ = ctx.prove_raw(wtns, bls[0])
    assert proof.hex() == meta["proofs"]["fixed"]["proof_bin"]
    ctx.set_lanes(1)
    assert ctx.lanes == 1


def test_batch_reports_lowest_failing_index():
    meta, zkey, wtns = _gold("p8")
    w = binfmt.read_wtns(wtns)["witness"]
    good = b"".join(x.to_bytes(32, "little") for x in w)
    w[20] = w[20] + 1
    bad = b"".join(x.to_bytes(32, "little") for x in w)
    ctx = nzcb.ProverContext(zkey)
    ctx.set_lanes(2)
    with pytest.raises(nzcb.NzcbError) as ei:
        ctx.prove_batch_raw([good, good, bad, good, bad])
    assert str(ei.value) == "proof 2: T Polynomial is not divisible"


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_msm_split_over_devices_bit_exact(devices):
    """commitment MSMs split by point range over several
    devices (here the same device several times: the partition, the peer copies and the
    host-side sum of partials are exercised) give the golden proof bits."""
    meta, zkey, wtns = _gold("p8")
    ctx = nzcb.ProverContext(zkey)
    ctx.set_msm_devices(devices)
    for bl in ("fixed", "zero"):
        exp = meta["proofs"][bl]
        blinding = bytes.fromhex(exp["blinding"]) if exp["blinding"] else bytes(352)  # explicit zero blinding
        proof, _ = ctx.prove_raw(wtns, blinding)
        assert proof.hex() == exp["proof_bin"]
    ctx.set_msm_devices([0])
    proof, _ = ctx.prove_raw(wtns, bytes.fromhex(meta["proofs"]["fixed"]["blinding"]))
    assert proof.hex() == meta["proofs"]["fixed"]["proof_bin"]
    with pytest.raises(nzcb.NzcbError):
        ctx.set_msm_devices([1 if nzcb.device_count() > 1 else 5, 0])


def test_msm_split_live_oracle():
    c = synth.synth_circuit(10, 3, 8, seed=41)
    zk = plonk.setup(c, 99991)
    from oracle.bn254 import R_MOD
    bl = [(41 * 7919 + i * 104729 + (i << 200)) % R_MOD for i in range(11)]
    proof, pub = plonk.prove(zk, c["witness"], bl)
    ctx = nzcb.ProverContext(binfmt.write_zkey(zk))
    ctx.set_msm_devices([0, 0, 0, 0])
    got, _ = ctx.prove_raw(binfmt.write_wtns(c["witness"]), b"".join(x.to_bytes(32, "little") for x in bl))
    assert got == plonk.proof_to_bytes(proof)


@pytest.mark.parametrize("quot3,lcommit", [("0", "1"), ("1", "1"), ("1", "0")])
def test_quotient_schedules_same_proof(quot3, lcommit):
    """The three-coset quotient (default, n >= 64) and the 4n coset one (NZCB_QUOT3=0; also
    every n < 64, e.g. p5 above) prove p8 bit for bit, and both report a broken gate as
    snarkjs's "T Polynomial is not divisible" (a fresh process: the switch is read once).
    Under the three-coset quotient the gate check runs on round 1's side stream with the
    Lagrange-basis commitments (default) and in round 3 without them
    (NZCB_LAGRANGE_COMMIT=0); after the error the context proves bit for bit again."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = (
        "import sys, json; sys.path[:0] = [%r, %r]\n"
        "import nzcb\n"
        "from oracle import binfmt\n"
        "g = %r\n"
        "meta = json.load(open(g + '/p8.json')); exp = meta['proofs']['fixed']\n"
        "zkey = open(g + '/p8.zkey', 'rb').read(); wtns = open(g + '/p8.wtns', 'rb').read()\n"
        "ctx = nzcb.ProverContext(zkey)\n"
        "proof, _ = ctx.prove_raw(wtns, bytes.fromhex(exp['blinding']))\n"
        "assert proof.hex() == exp['proof_bin'], 'proof differs'\n"
        "w = binfmt.read_wtns(wtns)['witness']; w[20] = w[20] + 1\n"
        "try:\n"
        "    ctx.prove_raw(binfmt.write_wtns(w)); raise SystemExit('no error')\n"
        "except nzcb.NzcbError as e:\n"
        "    assert str(e) == 'T Polynomial is not divisible', str(e)\n"
        "proof, _ = ctx.prove_raw(wtns, bytes.fromhex(exp['blinding']))\n"
        "assert proof.hex() == exp['proof_bin'], 'proof differs after the error'\n"
        "print('ok')\n" % (os.path.join(root, "nzcb-circom_amd"), root, GOLD))
    env = dict(os.environ, NZCB_QUOT3=quot3, NZCB_LAGRANGE_COMMIT=lcommit)
    p = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0 and p.stdout.strip().endswith("ok"), p.stdout + p.stderr


@pytest.mark.parametrize("sparse,sets", [("0", "0"), ("0", "1"), ("1", "0"), ("1", "1")])
def test_abc_commitment_schedules_same_proof(sparse, sets):
    """Round 6's two switches of the A, B, C commitments, both sides each (a fresh process:
    they are read once): NZCB_SPARSE (the Lagrange table's device-derived chunk and carry
    trees) and NZCB_ABC_SETS (the three commitments as one 3-set MSM instead of three). p5
    and p8 prove bit for bit, on one lane and on three lanes at once."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = (
        "import sys, json; sys.path[:0] = [%r, %r]\n"
        "import nzcb\n"
        "from oracle import binfmt\n"
        "g = %r\n"
        "for name in ('p5', 'p8'):\n"
        "    meta = json.load(open(g + '/' + name + '.json')); exp = meta['proofs']['fixed']\n"
        "    zkey = open(g + '/' + name + '.zkey', 'rb').read(); wtns = open(g + '/' + name + '.wtns', 'rb').read()\n"
        "    wit = b''.join(x.to_bytes(32, 'little') for x in binfmt.read_wtns(wtns)['witness'])\n"
        "    ctx = nzcb.ProverContext(zkey)\n"
        "    for lanes in (1, 3):\n"
        "        ctx.set_lanes(lanes)\n"
        "        res = ctx.prove_batch_raw([wit] * lanes, blindings=[bytes.fromhex(exp['blinding'])] * lanes)\n"
        "        assert all(p.hex() == exp['proof_bin'] for p, _ in res), (name, lanes)\n"
        "    ctx.close()\n"
        "print('ok')\n" % (os.path.join(root, "nzcb-circom_amd"), root, GOLD))
    env = dict(os.environ, NZCB_SPARSE=sparse, NZCB_ABC_SETS=sets)
    p = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0 and p.stdout.strip().endswith("ok"), p.stdout + p.stderr


@pytest.mark.parametrize("name", ["p5", "p8"])
def test_quotient_fault_is_caught_then_proves_again(name):
    """the xi check (prover.hip, round 4) is the only check on the
    three-coset t (p8; p5's n < 64 takes the 4n coset). A one-coefficient fault injected
    into t after round 3 is reported as NZCB_ERR_INTERNAL "quotient check failed", and the
    context's next proof is bit-exact again."""
    meta, zkey, wtns = _gold(name)
    exp = meta["proofs"]["fixed"]
    bl = bytes.fromhex(exp["blinding"])
    ctx = nzcb.ProverContext(zkey)
    try:
        ctx.inject_fault(nzcb.NZCB_FAULT_QUOTIENT)
        with pytest.raises(nzcb.NzcbError) as ei:
            ctx.prove_raw(wtns, bl)
        assert ei.value.name == "INTERNAL"
        assert str(ei.value).startswith("quotient check failed")
        proof, _ = ctx.prove_raw(wtns, bl)
        assert proof.hex() == exp["proof_bin"]
        ctx.inject_fault(0)   # set and cleared: nothing fires
        proof, _ = ctx.prove_raw(wtns, bl)
        assert proof.hex() == exp["proof_bin"]
    finally:
        ctx.close()
    ctx = nzcb.ProverContext(zkey)
    try:
        with pytest.raises(ValueError):
            ctx.inject_fault(7)
    finally:
        ctx.close()


@pytest.mark.parametrize("name", ["p5", "p8"])
def test_grand_product_generic_k_path_same_proof(name):
    """k_perm_tile forms k1 beta w^i and k2 beta w^i by their own Shoup products when k1, k2
    are not snarkjs' 2, 3 (prover.hip, round 2); nzcb_debug_inject_fault(NZCB_DEBUG_GENERIC_K)
    forces that path for one proof, which must still be the golden proof bit for bit, and so
    must the next one (one-shot)."""
    meta, zkey, wtns = _gold(name)
    exp = meta["proofs"]["fixed"]
    bl = bytes.fromhex(exp["blinding"])
    ctx = nzcb.ProverContext(zkey)
    try:
        ctx.inject_fault(nzcb.NZCB_DEBUG_GENERIC_K)
        proof, _ = ctx.prove_raw(wtns, bl)
        assert proof.hex() == exp["proof_bin"]
        proof, _ = ctx.prove_raw(wtns, bl)
        assert proof.hex() == exp["proof_bin"]
    finally:
        ctx.close()


def test_guard_words_selftest_and_lane_buffers():
    """The guard words behind every context buffer (common.h GuardScope): a one-word
    overrun past a fresh guarded buffer is found, and after proofs on 3 lanes and a lane
    count change every guard is intact."""
    nzcb.guard_selftest(0)
    meta, zkey, wtns = _gold("p8")
    exp = meta["proofs"]["fixed"]
    ctx = nzcb.ProverContext(zkey)
    try:
        ctx.set_lanes(3)
        wit = b"".join(x.to_bytes(32, "little") for x in binfmt.read_wtns(wtns)["witness"])
        res = ctx.prove_batch_raw([wit] * 6, blindings=[bytes.fromhex(exp["blinding"])] * 6)
        assert all(p.hex() == exp["proof_bin"] for p, _ in res)
        ctx.set_lanes(2)
        assert nzcb.guard_check(0) > 0
    finally:
        ctx.close()


def test_serial_profiling_mode_same_proof():
    """NZCB_SERIAL (profiling: every commitment MSM synchronised as it is enqueued) proves p8
    bit for bit in a fresh process, as the default does (test_golden_proof_bits)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = (
        "import sys, json; sys.path[:0] = [%r, %r]\n"
        "import nzcb\n"
        "g = %r\n"
        "meta = json.load(open(g + '/p8.json')); exp = meta['proofs']['fixed']\n"
        "zkey = open(g + '/p8.zkey', 'rb').read(); wtns = open(g + '/p8.wtns', 'rb').read()\n"
        "ctx = nzcb.ProverContext(zkey)\n"
        "proof, _ = ctx.prove_raw(wtns, bytes.fromhex(exp['blinding']))\n"
        "assert proof.hex() == exp['proof_bin'], 'proof differs'\n"
        "print('ok')\n" % (os.path.join(root, "nzcb-circom_amd"), root, GOLD))
    env = dict(os.environ, NZCB_SERIAL="1")
    p = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0 and p.stdout.strip().endswith("ok"), p.stdout + p.stderr


def test_failed_lane_growth_rolls_back_then_proves():
    """nzcb_ctx_set_lanes' rollback after a failed growth. NZCB_FAULT_LANE_ALLOC
    makes the next growth fail after its first new lane with a real failed hipMalloc (HIP's
    per-thread last error holds the out-of-memory code, as after a real one). The call
    raises, lanes stays at its old count, and on the same thread the next proofs (one lane,
    then a batch over the old lanes) are the golden proof bit for bit: the stale error was
    cleared. A later growth succeeds."""
    meta, zkey, wtns = _gold("p8")
    exp = meta["proofs"]["fixed"]
    bl = bytes.fromhex(exp["blinding"])
    wit = b"".join(x.to_bytes(32, "little") for x in binfmt.read_wtns(wtns)["witness"])
    ctx = nzcb.ProverContext(zkey)
    try:
        ctx.set_lanes(2)
        ctx.inject_fault(nzcb.NZCB_FAULT_LANE_ALLOC)
        with pytest.raises(nzcb.NzcbError) as ei:
            ctx.set_lanes(4)
        assert ei.value.name == "HIP" and "injected lane allocation failure" in str(ei.value)
        assert ctx.lanes == 2
        proof, _ = ctx.prove_raw(wtns, bl)
        assert proof.hex() == exp["proof_bin"]
        res = ctx.prove_batch_raw([wit] * 4, blindings=[bl] * 4)
        assert all(p.hex() == exp["proof_bin"] for p, _ in res)
        ctx.set_lanes(4)   # one-shot: the next growth goes through
        assert ctx.lanes == 4
        res = ctx.prove_batch_raw([wit] * 4, blindings=[bl] * 4)
        assert all(p.hex() == exp["proof_bin"] for p, _ in res)
        assert nzcb.guard_check(0) > 0
    finally:
        ctx.close()
