"""nzcb_synth_setup (GPU) emits the same zkey / wtns bytes as the CPU oracle's
synth_circuit + plonk.setup + binfmt writers (oracle/synth.py, oracle/plonk.py)."""
import pytest

import nzcb
from oracle import binfmt, plonk, synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("power,npub,nin,seed,ncons", [(4, 1, 2, 5, 0), (6, 3, 4, 6, 0), (8, 3, 8, 7, 200),
                                                       (9, 0, 3, 8, 0)])
def test_synth_setup_bytes(power, npub, nin, seed, ncons):
    tau = 0x1234567 + seed
    zkey, wtns = nzcb.synth_setup(power, npub, nin, seed, ncons, tau)
    c = synth.synth_circuit(power, npub, nin, seed=seed, n_constraints=ncons or None)
    zk = plonk.setup(c, tau)
    assert wtns == binfmt.write_wtns(c["witness"])
    assert zkey == binfmt.write_zkey(zk)


def test_synth_setup_proves_and_verifies():
    tau = 777
    zkey, wtns = nzcb.synth_setup(12, 3, 8, 99, 0, tau)
    ctx = nzcb.ProverContext(zkey)
    bl = b"".join(x.to_bytes(32, "little") for x in synth.fixed_blindings())
    proof, pub = ctx.prove_raw(wtns, bl)
    zk = binfmt.read_zkey(zkey)
    p = plonk.proof_from_bytes(proof)
    pubv = [int.from_bytes(pub[i:i + 32], "little") for i in range(0, len(pub), 32)]
    assert plonk.verify_with_trapdoor(zk, pubv, p, tau)


def test_full_pipeline_proofs_verify_with_pairing():
    """Larger synthetic circuit (2^14): random-blinding proofs from a 2-lane batch are
    accepted by the pairing verifier; a tampered one is rejected (size-independent
    parity check used by bench.py at 2^21)."""
    import nzcb
    ctx, wtns = nzcb.synth_context(14, 3, 40, seed=5, tau=0x1234567)
    nwit = (len(wtns) - 76) // 32
    wit = wtns[76:76 + 32 * nwit]
    ctx.set_lanes(2)
    res = ctx.prove_batch_raw([wit] * 3, blindings=[nzcb.random_blinding() for _ in range(3)])
    assert len({p for p, _ in res}) == 3
    for proof, pub in res:
        assert nzcb.verify(ctx.vk, proof, pub)
    bad = bytearray(res[0][0])
    bad[-1] ^= 1
    assert not nzcb.verify(ctx.vk, bytes(bad), res[0][1])


def test_batch_reports_failed_proofs_per_item():
    """in a batch, a witness that breaks the circuit fails its own proof
    only (nzcb_prove_batch_status); the plain batch call raises snarkjs's error."""
    import nzcb
    ctx, wtns = nzcb.synth_context(10, 3, 8, seed=9, tau=0x1234567)
    nwit = (len(wtns) - 76) // 32
    wit = wtns[76:76 + 32 * nwit]
    bad = bytearray(wit)
    bad[32 * (nwit - 1)] ^= 1
    bad = bytes(bad)
    ctx.set_lanes(2)
    st = []
    res = ctx.prove_batch_raw([wit, bad, wit, bad, wit], blindings=[nzcb.random_blinding() for _ in range(5)],
                              statuses=st)
    assert [s != 0 for s in st] == [False, True, False, True, False]
    assert st[1] == st[3] == 7  # NZCB_ERR_T_DIV
    assert res[1][0] == bytes(nzcb.PROOF_BYTES) and res[3][1] == bytes(len(res[3][1]))
    for i in (0, 2, 4):
        assert nzcb.verify(ctx.vk, res[i][0], res[i][1])
    with pytest.raises(nzcb.NzcbError, match="T Polynomial is not divisible"):
        ctx.prove_batch_raw([wit, bad])
