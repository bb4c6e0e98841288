"""Single-proof MSM split (configs[4]) and device-set contexts
(SURVEY.md §8b nzcb_ctx_create(devices)) on the GPU:

* nzcb_ctx_set_msm_split's callbacks, driven in one process: rank 0's own point range on
  the context, the other ranks' ranges on resident nzcb_msm_table tables of the same
  device (the work nzcb.msmsplit.serve does on each rank). The proofs equal the golden
  fixtures bit for bit, for 2, 3 and 5 ranks, and the batch entry points still work;
* nzcb_msm_table: the range partials add up to the unsplit MSM;
* the in-process split and a device-set batch over two distinct GPUs, where present
  (skipped on a one-GPU box).
The multi-process protocol itself (broadcast / all-gather over torch.distributed) is
covered over gloo in tests/test_dist.py."""
import json
import os

import pytest

from oracle import binfmt

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


class _Ptr:
    def __init__(self, p):
        self.p = p

    def data_ptr(self):
        return self.p


def msmsplit_counts(count, ranges):
    from nzcb import msmsplit
    return msmsplit.slice_counts(count, ranges)


class _LocalRanks:
    """The serving ranks of msmsplit, in-process: each range's partial is computed from a
    private copy of the scalars as soon as they are sent (as serve() does on its GPU)."""

    def __init__(self, nzcb, msmsplit, zkey, n_points: int, world: int):
        """zkey: bytes, or a (pointer, length) library buffer (nzcb.plonk_setup_raw)."""
        self.nzcb = nzcb
        if isinstance(zkey, tuple):
            addr, ln = msmsplit.zkey_section(zkey[0], zkey[1], 14)   # PTau [tau^i]G1
            self.ptau = nzcb.dev_alloc(ln)
            nzcb.memcpy_h2d_ptr(self.ptau, addr, ln)
        else:
            _, sec = binfmt.read_binfile(zkey, b"zkey")
            (o, ln), = sec[14]
            self.ptau = nzcb.dev_alloc(ln)
            nzcb.h2d(self.ptau, zkey[o:o + ln])
        self.ranges = msmsplit.point_ranges(n_points, world)
        self.backends = [msmsplit.GpuRange(self.ptau, lo, hi, 0) for lo, hi in self.ranges[1:]]
        self.scal = nzcb.dev_alloc(32 * n_points)
        self.pending = {}
        self.calls = 0

    def send(self, slot, ptr, count):
        self.nzcb.d2d(self.scal, ptr, 32 * count)
        cnts = msmsplit_counts(count, self.ranges)
        self.pending[slot] = b"".join(b(slot, _Ptr(self.scal + 32 * lo), c)
                                      for b, (lo, _), c in zip(self.backends, self.ranges[1:], cnts[1:]))
        self.calls += 1

    def gather(self, slot, own):
        return own + self.pending.pop(slot)

    def close(self):
        for b in self.backends:
            b.close()
        self.nzcb.dev_free(self.ptau)
        self.nzcb.dev_free(self.scal)


@pytest.mark.parametrize("world", [2, 3, 5])
def test_msm_split_callbacks_bit_exact(world):
    import nzcb
    from nzcb import msmsplit
    meta, zkey, wtns = _gold("p8")
    ctx = nzcb.ProverContext(zkey)
    ranks = _LocalRanks(nzcb, msmsplit, zkey, ctx.domain_size + 6, world)
    try:
        ctx.set_msm_split(world, ranks.ranges[0][1], ranks.send, ranks.gather)
        for bl in ("fixed", "zero"):
            exp = meta["proofs"][bl]
            blinding = bytes.fromhex(exp["blinding"]) if exp["blinding"] else bytes(352)
            proof, _ = ctx.prove_raw(wtns, blinding)
            assert proof.hex() == exp["proof_bin"]
        # 6 split commitments per proof (A, B, C are committed locally in the Lagrange basis)
        per_proof = 9 if os.environ.get("NZCB_LAGRANGE_COMMIT") == "0" else 6
        assert ranks.calls == 2 * per_proof and not ranks.pending
        ctx.set_lanes(2)   # a split context proves its batches on lane 0
        w = binfmt.read_wtns(wtns)["witness"]
        wit = b"".join(x.to_bytes(32, "little") for x in w)
        res = ctx.prove_batch_raw([wit] * 3, blindings=[bytes.fromhex(meta["proofs"]["fixed"]["blinding"])] * 3)
        assert all(p.hex() == meta["proofs"]["fixed"]["proof_bin"] for p, _ in res)
        ctx.set_msm_split(1, 0, None, None)
        proof, _ = ctx.prove_raw(wtns, bytes.fromhex(meta["proofs"]["fixed"]["blinding"]))
        assert proof.hex() == meta["proofs"]["fixed"]["proof_bin"]
        with pytest.raises(nzcb.NzcbError):         # a gather that fails fails the proof
            ctx.set_msm_split(world, ranks.ranges[0][1], ranks.send, lambda slot, own: b"")
            ctx.prove_raw(wtns, bytes(352))
    finally:
        ranks.close()
        ctx.close()


def test_msm_table_ranges_add_up():
    import nzcb
    from nzcb import msmsplit
    from oracle import bn254 as bn
    n = 1 << 16
    eng = nzcb.Engine(0, max_log_ntt=-1, max_msm_points=n + 8)
    sc, bases = nzcb.dev_alloc(n * 32), nzcb.dev_alloc(n * 64)
    try:
        eng.random_fr(sc, n, 0x7AB1E)
        eng.fixed_base(sc, n, bases)
        eng.random_fr(sc, n, 0x5CA1)
        whole = eng.msm_dev(bases, sc, n, True)
        acc = None
        for lo, hi in msmsplit.point_ranges(n, 3):
            t = nzcb.MsmTable(bases + 64 * lo, hi - lo)
            p = t.run(sc + 32 * lo, hi - lo, True)
            t.close()
            x, y = bn.from_le(p[:32]), bn.from_le(p[32:])
            acc = bn.g1_add(acc, None if x == 0 and y == 0 else (x, y))
    finally:
        nzcb.dev_free(sc)
        nzcb.dev_free(bases)
        eng.close()
    assert acc == (bn.from_le(whole[:32]), bn.from_le(whole[32:]))


def test_two_distinct_devices_where_present():
    """the cross-device paths on two distinct device ids (peer copies of the
    scalar slices, a shard table in the other GPU's HBM; a device-set batch with witnesses
    in device 0's HBM read by device 1's lanes). Skipped with fewer than 2 GPUs."""
    import nzcb
    if nzcb.device_count() < 2:
        pytest.skip("needs two GPUs")
    meta, zkey, wtns = _gold("p8")
    bl = bytes.fromhex(meta["proofs"]["fixed"]["blinding"])
    ctx = nzcb.ProverContext(zkey)
    ctx.set_msm_devices([0, 1])
    proof, _ = ctx.prove_raw(wtns, bl)
    assert proof.hex() == meta["proofs"]["fixed"]["proof_bin"]
    ctx.close()
    ctx = nzcb.ProverContext(zkey, devices=[0, 1])
    ctx.set_lanes(2)
    w = binfmt.read_wtns(wtns)["witness"]
    wit = b"".join(x.to_bytes(32, "little") for x in w)
    dev = nzcb.dev_alloc(len(wit))
    try:
        nzcb.h2d(dev, wit)
        res = ctx.prove_batch_raw([dev] * 6, n_witness=len(w), blindings=[bl] * 6, on_device=True)
    finally:
        nzcb.dev_free(dev)
        ctx.close()
    assert all(p.hex() == meta["proofs"]["fixed"]["proof_bin"] for p, _ in res)


def test_device_set_context_single_device():
    """nzcb_ctx_create_devices with one id behaves as nzcb_ctx_create; a repeated id is
    rejected."""
    import nzcb
    meta, zkey, wtns = _gold("p5")
    ctx = nzcb.ProverContext(zkey, devices=[0])
    exp = meta["proofs"]["fixed"]
    proof, _ = ctx.prove_raw(wtns, bytes.fromhex(exp["blinding"]))
    assert proof.hex() == exp["proof_bin"]
    assert nzcb.load().nzcb_ctx_devices(ctx.h) == 1
    ctx.close()
    with pytest.raises(nzcb.NzcbError, match="appears twice"):
        nzcb.ProverContext(zkey, devices=[0, 0])
