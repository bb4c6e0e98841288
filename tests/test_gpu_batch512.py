"""BASELINE.json configs[3] ("Batch of 512 nzcp_live proofs sharded across 8 x MI355X,
embarrassingly parallel, no RCCL") as a -m gpu test on the one GPU a test box has: the 512
passes are cut into bench.py's 8 shards (bench.shard(512, r, 8)) and the shards are proved
one after another through the production path each rank runs (GPU witness program ->
nzcb_prove_batch over 5 lanes, nzcb/nzcplive.py NzcpLiveProver.full_prove_staged).

Checked: every one of the 512 proofs' public signals equals its pass's outputs from the
independent nzcp kernel (csrc/nzcp.hip, pinned by the reference's KATs); the 512 proofs are
distinct; each shard's first and last proof pass the pairing verifier; every guard word past
the context's device buffers is intact afterwards; shard 0's first proof is byte-equal to
the C port's (oracle/c/nzcb_ref.c) on the same zkey, GPU witness and blinding. What the
8-GPU run adds (8 processes, one GPU each, bench.py --gpus 8 --batch 512) is unmeasured here:
the shards share nothing, so each rank's work is exactly one of these loops."""
import pytest

pytestmark = pytest.mark.gpu


def _ints(raw):
    return [int.from_bytes(raw[i:i + 32], "little") for i in range(0, len(raw), 32)]


@pytest.mark.timeout(900)
def test_configs3_batch_512_in_8_shards():
    import bench
    import nzcb
    from nzcb import nzcplive
    from oracle import cbind
    r1cs, prog, _ = nzcplive.build()
    ctx, zkey = nzcplive.context(r1cs, bench.TAU)
    prover = nzcplive.NzcpLiveProver(ctx, prog)
    seen = set()
    first = None
    try:
        ctx.set_lanes(5)
        for rank in range(8):
            idx = list(bench.shard(512, rank, 8))
            assert len(idx) == 64
            inputs = bench.pass_inputs(idx)
            prover.upload_inputs(inputs)
            res = prover.full_prove_staged(len(idx), [bench.blinding_for(i) for i in idx])
            records = nzcb.nzcp_witness(inputs, len(idx), nzcb.NZCP_LIVE, ctx.device)
            assert len(res) == len(idx) == len(records)
            for (proof, pub), rec in zip(res, records):
                assert rec["status"] == 0
                assert _ints(pub) == rec["out"]
                seen.add(proof)
            for k in (0, len(res) - 1):
                assert nzcb.verify(ctx.vk, res[k][0], res[k][1]), (rank, k)
            if rank == 0:
                first = (res[0][0], res[0][1], prover.witness_bytes(0))
        assert len(seen) == 512
        assert nzcb.guard_check(ctx.device) > 0
    finally:
        prover.close()
        ctx.close()
    try:
        ref_proof, ref_pub, _ = cbind.prove(zkey, nzcplive.wtns_file(first[2]), bench.blinding_for(0), npub=3)
    finally:
        nzcb.free_ptr(zkey[0])
    assert first[0] == ref_proof and first[1] == ref_pub[:96]
