"""The GPU witness VM (csrc/wvm.hip) running the nzcp circuits' witness programs, and
fullProve of the real NZCPPubIdentity statement:

* every committed golden nzcp case (118 nzcp_live + the example pass on
  nzcp_example's program): status equal to the CPU restatement's (pinned by the
  reference's KATs), public outputs equal, and every wire of every witness bit-exact
  against the CPU evaluation of the program (oracle/wvm.py), for passing and failing
  passes alike; the GPU witnesses satisfy the r1cs;
* nzcp_live at full size: r1cs -> seeded ptau-21 -> nzcb_plonk_setup (2^21 domain) ->
  NzcpLiveProver.full_prove (GPU witness program -> nzcb_prove_batch): publics equal
  the restatement's outputs, the proofs pass the pairing check, and the proof bytes equal
  the C port's (oracle/c/nzcb_ref.c) on the same zkey, GPU witness and blinding.

Parity against snarkjs on circom's nzcp_live.zkey stays unpinned (nzcb/nzcpgen.py)."""
import json
import os

import pytest

import nzcp_cases as C
from oracle import nzcp_circuit as nz
from oracle import wvm

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "nzcp_cases.json")
R = nz.R_MOD


@pytest.fixture(scope="module")
def programs():
    from nzcb import nzcpgen
    out = {}
    for key, params in (("live", nzcpgen.LIVE), ("example", nzcpgen.EXAMPLE)):
        c = nzcpgen.nzcp_pub_identity(**params)
        out[key] = (c, c.write_program())
    return out


def _unsat(c, wit, limit=3):
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


def _ints(raw):
    return [int.from_bytes(raw[i:i + 32], "little") for i in range(0, len(raw), 32)]


def test_golden_cases_gpu_witness_bit_exact(programs):
    import nzcb
    with open(GOLD) as f:
        gold = json.load(f)
    groups = {}
    for case, exp in zip(gold["cases"], gold["expected"]):
        key = "live" if case["params"]["is_live"] else "example"
        groups.setdefault(key, []).append((case, exp))
    checked_r1cs = 0
    for key, items in groups.items():
        c, prog = programs[key]
        wp = nzcb.WitnessProgram(prog)
        try:
            inputs = b"".join(C.case_input_bytes(case) for case, _ in items)
            raw, st = wp.run(inputs, len(items))
        finally:
            wp.close()
        stride = c.n_wires * 32
        for i, (case, exp) in enumerate(items):
            got = _ints(raw[i * stride:(i + 1) * stride])
            bits, ln, data = C.case_signals(case)
            want, fail = wvm.evaluate(prog, bits + [ln] + data)
            assert st[i] == (fail[1] if fail else 0), case["name"]
            if exp["status"] == nz.ERR_UNPINNED:  # negative length: the circuit's range check rejects it
                assert st[i] == nz.ERR_RANGE, case["name"]
            else:
                assert st[i] == exp["status"], case["name"]
            assert got == want, case["name"]
            if exp["status"] == 0:
                assert got[1:4] == [int(v) for v in exp["out"]], case["name"]
                if checked_r1cs < 3:
                    assert _unsat(c, got) == [], case["name"]
                    checked_r1cs += 1
    assert sum(len(v) for v in groups.values()) == len(gold["cases"])


@pytest.mark.timeout(900)
def test_nzcp_live_full_prove_real_circuit():
    import nzcb
    from nzcb import nzcplive
    from oracle import cbind, synth
    r1cs, prog, _ = nzcplive.build()
    ctx, zkey = nzcplive.context(r1cs)
    assert ctx.domain_size == 1 << 21 and ctx.n_public == 3
    prover = nzcplive.NzcpLiveProver(ctx, prog)
    cases = [C.case(f"p{i}", nz.LIVE_PARAMS, C.live_tbs(subject=C.credential_subject(g, f, d)),
                    data=bytes([i + 1]) * 20)
             for i, (g, f, d) in enumerate((("Jack", "Sparrow", "1960-04-16"), ("Jo", "Bloggs", "1999-12-31")))]
    bl = b"".join(x.to_bytes(32, "little") for x in synth.fixed_blindings())
    try:
        ctx.set_lanes(2)
        res = prover.full_prove(b"".join(C.case_input_bytes(cs) for cs in cases), [bl, bl])
        wit0 = prover.witness_bytes(0)
        with pytest.raises(nzcb.NzcbError):
            prover.full_prove(C.case_input_bytes(C.case("bad", nz.LIVE_PARAMS, C.live_tbs(), length=360)))
    finally:
        prover.close()
    for case, (proof, pub) in zip(cases, res):
        exp = [int(v) for v in C.oracle_record(case)["out"]]
        assert _ints(pub) == exp
        assert nzcb.verify(ctx.vk, proof, pub)
    assert res[0][0] != res[1][0]
    # the generated Solidity verifier (zkey export solidityverifier) accepts the real
    # statement's proof, executed by tests/yul.py on the calldata's proof bytes
    from tests import yul
    sol = nzcb.vk_to_solidity(ctx.vk, "Verifier")
    words = bytes.fromhex(nzcb.proof_to_calldata(res[0][0], b"").split(",")[0][2:])
    assert yul.run_verify_proof(sol, words, _ints(res[0][1]))[0]
    # configs[4] on one GPU: every commitment divided into 8 point ranges (PTau for Z, T1..T3,
    # Wxi, Wxiw; the Lagrange basis for A, B, C since round 6), ranks 1..7 served in-process
    # from resident range tables (what msmsplit.serve does per GPU), the partials folded in
    # rank order; the proof must not change by a bit
    from nzcb import msmsplit
    from tests.test_gpu_split import _LocalRanks
    # bucket entries of one proof (kernel statistics): six dense MSMs at 13 per scalar plus
    # A, B, C in the Lagrange basis bucketed as min(s, r - s) (msm.hip scalar_min_form): about
    # 2.2 n for the three (21.7 M, 10.3 n, before round 6's sign flip)
    n = ctx.domain_size
    ctx.set_lanes(1)
    ctx.kernel_stats(1)
    assert ctx.prove_witness_raw(wit0, bl)[0] == res[0][0]
    _, launches, _, entries = ctx.kernel_stats(0)
    dense = 6 * 13 * (n + 6)
    assert launches == 7 and dense - n < entries < dense + 3 * n, (launches, entries)
    ranks = _LocalRanks(nzcb, msmsplit, zkey, ctx.domain_size + 6, 8)
    try:
        ctx.set_lanes(1)
        ctx.set_msm_split(8, ranks.ranges[0][1], ranks.send, ranks.gather, ranks.own_lagrange)
        split_proof, split_pub = ctx.prove_witness_raw(wit0, bl)
        ctx.set_msm_split(1, 0, None, None)
        assert ranks.calls == 9 and ranks.lagrange_calls == 3 and not ranks.pending   # all nine commitments
    finally:
        ranks.close()
    ctx.close()
    try:
        ref_proof, ref_pub, _ = cbind.prove(zkey, nzcplive.wtns_file(wit0), bl, npub=3)
    finally:
        nzcb.free_ptr(zkey[0])
    assert res[0][0] == ref_proof and res[0][1] == ref_pub[:96]
    assert split_proof == ref_proof and split_pub == res[0][1]


def test_remapped_programs_on_gpu():
    """nzcb_wprog_remap on the GPU: programs re-indexed to a permuted
    .sym (tests/test_wprog_remap.py permuted_sym) write their witnesses in the target order.
    * NZCPPubIdentity(1, 351, 0, 4, 2, 4), all 600,560 signals of a live pass: every wire
      equals the CPU evaluation of the original program, moved to its target index;
    * a reference test main (skipValue5_test): the remapped GPU witness proves against a
      zkey set up from the r1cs written in the permuted order, byte-equal to the C port's
      proof of the CPU witness on the same zkey and blinding.
    Parity of the names with circom's own nzcp_live.sym stays unpinned."""
    import nzcb
    from nzcb import nzcpgen, nzcplive
    from oracle import cbind, synth
    from tests.test_wprog_remap import permuted_sym
    c = nzcpgen.nzcp_pub_identity(**nzcpgen.LIVE)
    prog = c.write_program()
    sym, new = permuted_sym(c, 0x5E)
    mapped = nzcb.wprog_remap(prog, c.write_sym(), sym)
    case = C.case("live", nz.LIVE_PARAMS, C.live_tbs(), data=bytes(range(1, 21)))
    wp = nzcb.WitnessProgram(mapped)
    try:
        assert wp.n_wires == c.n_wires
        raw, st = wp.run(C.case_input_bytes(case), 1)
    finally:
        wp.close()
    assert st == [0]
    got = _ints(raw)
    bits, ln, data = C.case_signals(case)
    want, fail = wvm.evaluate(prog, bits + [ln] + data)
    assert fail is None and got[0] == 1
    assert all(got[new[k]] == want[k] for k in range(1, c.n_wires))
    # a small main end to end: remapped GPU witness -> proof over the permuted r1cs
    g = nzcpgen.wrapper_circuit("skipValue5_test")
    gsym, gnew = permuted_sym(g, 0x5F)
    gmapped = nzcb.wprog_remap(g.write_program(), g.write_sym(), gsym)
    zkey = nzcb.plonk_setup(g.write_r1cs(gnew), nzcb.ptau_synth(12, 0x6E7A6362746175))
    inputs = [0x83, 0x61, 0x71, 0x17, 0x17, 0]              # [\"q\", 23, 23]: nextPos 5
    wp = nzcb.WitnessProgram(gmapped)
    try:
        raw, st = wp.run(b"".join(v.to_bytes(32, "little") for v in inputs), 1)
    finally:
        wp.close()
    gw, gfail = wvm.evaluate(gmapped, inputs)
    assert st == [0] and gfail is None and _ints(raw) == gw and gw[gnew[1]] == 5
    bl = b"".join(x.to_bytes(32, "little") for x in synth.fixed_blindings())
    ctx = nzcb.ProverContext(zkey)
    try:
        proof, pub = ctx.prove_witness_raw(raw, bl)
        assert nzcb.verify(ctx.vk, proof, pub)
    finally:
        ctx.close()
    ref_proof, ref_pub, _ = cbind.prove(zkey, nzcplive.wtns_file(raw), bl, npub=1)
    assert proof == ref_proof and pub == ref_pub[:32]


def test_level_clock_probe_same_witness(programs, tmp_path):
    """NZCB_WVM_LEVEL_CLOCK (tools/wvm_bench.py --levels): with the per-level clock on, the
    example pass's witness is the one computed without it, and the clock file holds one
    record block per level (fresh process: the switch is read at the run)."""
    import subprocess
    import sys
    import nzcb
    c, prog = programs["example"]
    gold = json.load(open(GOLD))
    case = next(cs for cs in gold["cases"] if not cs["params"]["is_live"])
    inputs = C.case_input_bytes(case)
    pp, ip, op = tmp_path / "p.nzwp", tmp_path / "in.bin", tmp_path / "w.bin"
    pp.write_bytes(prog)
    ip.write_bytes(inputs)
    wp = nzcb.WitnessProgram(prog)
    try:
        want, st = wp.run(inputs, 1)
        n_levels = wp.n_levels
    finally:
        wp.close()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    clock = tmp_path / "clock.bin"
    script = ("import sys; sys.path[:0] = [%r]\n"
              "import nzcb\n"
              "wp = nzcb.WitnessProgram(open(%r, 'rb').read())\n"
              "raw, st = wp.run(open(%r, 'rb').read(), 1)\n"
              "open(%r, 'wb').write(raw)\n"
              "print('ok', list(st))\n" % (os.path.join(root, "nzcb-circom_amd"), str(pp), str(ip), str(op)))
    p = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, NZCB_WVM_LEVEL_CLOCK=str(clock)))
    assert p.returncode == 0 and "ok" in p.stdout, p.stdout + p.stderr
    assert f"ok {list(st)}" in p.stdout
    assert op.read_bytes() == want
    size = clock.stat().st_size
    assert size > 0 and size % (8 * (n_levels + 1)) == 0
