"""R1CS -> PLONK setup (snarkjs `plonk setup <r1cs> <ptau>`, /root/reference/Makefile:55,60).

CPU: the restatement of processConstraints (oracle/r1cs.py) on hand-checked gates and on
seeded satisfiable r1cs files (every PLONK gate holds on the extended witness).
GPU: nzcb_plonk_setup (csrc/synth.hip) emits the oracle's zkey bytes, and the zkey
proves and verifies. Parity against snarkjs itself is unpinned (no reference r1cs,
ptau or zkey files exist)."""
import pytest

from oracle import binfmt, plonk, r1cs
from oracle.bn254 import R_MOD


def _gate_holds(g, w):
    a, b, c = w[g[0]], w[g[1]], w[g[2]]
    qm, ql, qr, qo, qc = g[3:]
    return (qm * a * b + ql * a + qr * b + qo * c + qc) % R_MOD == 0


def test_reduce_coef_order_and_gates():
    # out1 = 7 (2 w2 + 3 w3 + 5 w4); wires: 0 one, 1 out, 2 pub in, 3-4 private
    A = [(2, 2), (3, 3), (4, 5)]
    B = [(0, 7)]
    C = [(1, 1)]
    data = r1cs.write_r1cs(5, 1, 1, 2, [(A, B, C)])
    rc = r1cs.read_r1cs(data)
    assert rc["nWires"] == 5 and rc["constraints"] == [(A, B, C)] and rc["prime"] == R_MOD
    c = r1cs.process_constraints(rc)
    neg = lambda v: -v % R_MOD  # noqa: E731
    assert c["nPublic"] == 2 and c["nVars"] == 7 and c["nAdditions"] == 2 and c["power"] == 3
    assert c["constraints"] == [
        [1, 0, 0, 0, 1, 0, 0, 0],
        [2, 0, 0, 0, 1, 0, 0, 0],
        [3, 4, 5, 0, neg(3), neg(5), 1, 0],   # second half first folded: w5 = 3 w3 + 5 w4
        [2, 5, 6, 0, neg(2), neg(1), 1, 0],   # w6 = 2 w2 + 1 w5
        [6, 0, 1, 0, 7, 0, neg(1), 0],        # (w6)(7) = w1
    ]
    assert c["additions"] == [(3, 4, 3, 5), (2, 5, 2, 1)]
    w = [1, 0, 11, 13, 17]
    w[1] = 7 * (2 * 11 + 3 * 13 + 5 * 17) % R_MOD
    ext = r1cs.extend_witness(c, w)
    assert all(_gate_holds(g, ext) for g in c["constraints"][c["nPublic"]:])  # PI rows: ql a + PI = 0


@pytest.mark.parametrize("nc,power", [(1, 3), (8, 3), (9, 4), (16, 4), (17, 5), (1025, 11)])
def test_domain_power(nc, power):
    """cirPower = log2(nConstraints - 1) + 1 (floor log2), at least 3."""
    cons = [([(1, 1)], [(0, 1)], [(1, 1)])] * (nc - 1)   # plus the one public gate
    c = r1cs.process_constraints(r1cs.read_r1cs(r1cs.write_r1cs(2, 1, 0, 0, cons)))
    assert len(c["constraints"]) == nc and c["power"] == power


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_r1cs_satisfied_after_processing(seed):
    data, w = r1cs.random_r1cs(seed)
    rc = r1cs.read_r1cs(data)
    for A, B, C in rc["constraints"]:
        val = lambda lc: sum(c * w[s] for s, c in lc) % R_MOD  # noqa: E731
        assert val(A) * val(B) % R_MOD == val(C)
    c = r1cs.process_constraints(rc)
    ext = r1cs.extend_witness(c, w)
    assert len(ext) == c["nVars"]
    assert all(_gate_holds(g, ext) for g in c["constraints"][c["nPublic"]:])
    used = {s for g in c["constraints"] for s in g[:3]}
    assert used == set(range(c["nVars"]))   # else snarkjs throws "Variable not used"


TAU = 0x5E7A9
_PTAU = {}


def _ptau(power):
    if power not in _PTAU:
        _PTAU[power] = r1cs.write_ptau(TAU, power)
    return _PTAU[power]


@pytest.mark.gpu
@pytest.mark.parametrize("seed,steps", [(11, 12), (12, 40), (13, 90)])
def test_plonk_setup_bytes_match_oracle(seed, steps):
    import nzcb
    data, _ = r1cs.random_r1cs(seed, n_steps=steps)
    c = r1cs.process_constraints(r1cs.read_r1cs(data))
    zkey = nzcb.plonk_setup(data, _ptau(9))
    assert zkey == binfmt.write_zkey(plonk.setup(c, TAU))


@pytest.mark.gpu
def test_plonk_setup_zkey_proves_and_verifies():
    """The r1cs zkey through the GPU prover: bit-exact against the C oracle prover with
    fixed blinding, accepted by the pairing verifier and by the trapdoor check."""
    import nzcb
    from oracle import cbind, synth
    data, w = r1cs.random_r1cs(21, n_out=3, n_pub_in=2, n_prv_in=4, n_steps=120)
    zkey = nzcb.plonk_setup(data, _ptau(9))
    wtns = binfmt.write_wtns(w)
    bl = b"".join(x.to_bytes(32, "little") for x in synth.fixed_blindings())
    ctx = nzcb.ProverContext(zkey)
    try:
        proof, pub = ctx.prove_raw(wtns, bl)
        assert nzcb.verify(ctx.vk, proof, pub)
    finally:
        ctx.close()
    assert [int.from_bytes(pub[i:i + 32], "little") for i in range(0, len(pub), 32)] == w[1:6]
    ref_proof, ref_pub, _ = cbind.prove(zkey, wtns, bl)
    assert proof == ref_proof and pub == ref_pub[:len(pub)]
    zk = binfmt.read_zkey(zkey)
    assert plonk.verify_with_trapdoor(zk, w[1:6], plonk.proof_from_bytes(proof), TAU)


@pytest.mark.gpu
def test_plonk_setup_errors():
    import nzcb
    data, _ = r1cs.random_r1cs(5, n_steps=90)   # 2^7 domain
    with pytest.raises(nzcb.NzcbError, match="circuit too big for this power of tau ceremony"):
        nzcb.plonk_setup(data, _ptau(3))
    bad = bytearray(data)
    off = data.index(R_MOD.to_bytes(32, "little"))
    bad[off] ^= 1
    with pytest.raises(nzcb.NzcbError, match="r1cs curve does not match"):
        nzcb.plonk_setup(bytes(bad), _ptau(9))
    with pytest.raises(nzcb.NzcbError, match="invalid file format"):
        nzcb.plonk_setup(b"junk" + data[4:], _ptau(9))


@pytest.mark.gpu
def test_plonk_setup_larger_circuit_proves_and_verifies():
    """A 2^15-domain r1cs (5000 constraints folded into about 18.9k PLONK gates) against a
    2^15 ptau whose tauG1 points come from the GPU fixed-base kernel: the zkey proves
    and the pairing verifier accepts (size-independent check of the setup's
    commitments), and the proof equals the C oracle prover's on the same zkey."""
    import nzcb
    import struct
    from oracle import bn254 as bn, cbind, synth
    from oracle.binfmt import write_binfile
    power = 15
    cnt = (1 << (power + 1)) - 1
    scal = bytearray()
    t = 1
    for _ in range(cnt):
        scal += bn.to_lem(t, R_MOD)
        t = t * TAU % R_MOD
    eng = nzcb.Engine(0, max_log_ntt=-1, max_msm_points=0)
    ds, dp = nzcb.dev_alloc(len(scal)), nzcb.dev_alloc(64 * cnt)
    try:
        nzcb.h2d(ds, bytes(scal))
        eng.fixed_base(ds, cnt, dp)
        g1 = nzcb.d2h(dp, 64 * cnt)
    finally:
        nzcb.dev_free(ds)
        nzcb.dev_free(dp)
        eng.close()
    assert bn.g1_from_lem(g1[64:128]) == bn.g1_mul(bn.G1_GEN, TAU)
    s1 = struct.pack("<I", 32) + bn.to_le(bn.P_MOD) + struct.pack("<II", power, power)
    g2 = bn.g2_to_lem(bn.G2_GEN) + bn.g2_to_lem(bn.g2_mul(bn.G2_GEN, TAU))
    ptau = write_binfile(b"ptau", 1, [(1, s1), (2, g1), (3, g2)])
    data, w = r1cs.random_r1cs(77, n_out=3, n_pub_in=1, n_prv_in=6, n_steps=5000)
    zkey = nzcb.plonk_setup(data, ptau)
    wtns = binfmt.write_wtns(w)
    bl = b"".join(x.to_bytes(32, "little") for x in synth.fixed_blindings())
    ctx = nzcb.ProverContext(zkey)
    try:
        assert ctx.domain_size == 1 << 15
        proof, pub = ctx.prove_raw(wtns, bl)
        assert nzcb.verify(ctx.vk, proof, pub)
    finally:
        ctx.close()
    ref_proof, ref_pub, _ = cbind.prove(zkey, wtns, bl)
    assert proof == ref_proof and pub == ref_pub[:len(pub)]
