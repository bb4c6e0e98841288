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
    private copy of the scalars as soon as they are sent (as serve() does on its GPU). PTau
    ranges for the six random-scalar commitments and, unless the context commits A, B, C
    from coefficients (NZCB_LAGRANGE_COMMIT=0), ranges of the n + 2-point Lagrange basis,
    computed on the GPU from the PTau (nzcb_msm_table_create_lagrange)."""

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
        self.msmsplit = msmsplit
        self.ranges = msmsplit.point_ranges(n_points, world)
        self.backends = [msmsplit.GpuRange(self.ptau, lo, hi, 0) for lo, hi in self.ranges[1:]]
        n = n_points - 6
        self.lranges, self.lbackends = None, []
        if nzcb.lagrange_commit_enabled():
            self.lranges = msmsplit.point_ranges(n + 2, world)
            self.lbackends = [msmsplit.GpuRange(self.ptau, lo, hi, 0, lagrange=True, ptau_n=n_points,
                                                log_n=n.bit_length() - 1) for lo, hi in self.lranges[1:]]
        self.own_lagrange = self.lranges[0][1] if self.lranges else 0
        self.scal = nzcb.dev_alloc(32 * n_points)
        self.pending = {}
        self.calls = 0
        self.lagrange_calls = 0

    def send(self, slot, ptr, count):
        slot, lag = self.msmsplit.split_slot(slot)
        ranges, backends = (self.lranges, self.lbackends) if lag else (self.ranges, self.backends)
        self.nzcb.d2d(self.scal, ptr, 32 * count)
        cnts = msmsplit_counts(count, ranges)
        self.pending[slot] = b"".join(b(slot, _Ptr(self.scal + 32 * lo), c)
                                      for b, (lo, _), c in zip(backends, ranges[1:], cnts[1:]))
        self.calls += 1
        self.lagrange_calls += lag

    def gather(self, slot, own):
        return own + self.pending.pop(self.msmsplit.split_slot(slot)[0])

    def close(self):
        for b in self.backends + self.lbackends:
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
        ctx.set_msm_split(world, ranks.ranges[0][1], ranks.send, ranks.gather, ranks.own_lagrange)
        for bl in ("fixed", "zero"):
            exp = meta["proofs"][bl]
            blinding = bytes.fromhex(exp["blinding"]) if exp["blinding"] else bytes(352)
            proof, _ = ctx.prove_raw(wtns, blinding)
            assert proof.hex() == exp["proof_bin"]
        # all 9 commitments per proof leave rank 0 (round 6: A, B, C over Lagrange-basis ranges)
        assert ranks.calls == 2 * 9 and not ranks.pending
        assert ranks.lagrange_calls == (0 if os.environ.get("NZCB_LAGRANGE_COMMIT") == "0" else 2 * 3)
        # own_lagrange = 0 keeps A, B, C on rank 0 (round 5's schedule): 6 split commitments
        ctx.set_msm_split(world, ranks.ranges[0][1], ranks.send, ranks.gather, 0)
        proof, _ = ctx.prove_raw(wtns, bytes.fromhex(meta["proofs"]["fixed"]["blinding"]))
        assert proof.hex() == meta["proofs"]["fixed"]["proof_bin"]
        assert ranks.calls == 2 * 9 + (9 if os.environ.get("NZCB_LAGRANGE_COMMIT") == "0" else 6)
        ctx.set_msm_split(world, ranks.ranges[0][1], ranks.send, ranks.gather, ranks.own_lagrange)
        ctx.set_lanes(2)   # a split context proves its batches on lane 0
        w = binfmt.read_wtns(wtns)["witness"]
        wit = b"".join(x.to_bytes(32, "little") for x in w)
        res = ctx.prove_batch_raw([wit] * 3, blindings=[bytes.fromhex(meta["proofs"]["fixed"]["blinding"])] * 3)
        assert all(p.hex() == meta["proofs"]["fixed"]["proof_bin"] for p, _ in res)
        ctx.set_msm_split(1, 0, None, None)
        proof, _ = ctx.prove_raw(wtns, bytes.fromhex(meta["proofs"]["fixed"]["blinding"]))
        assert proof.hex() == meta["proofs"]["fixed"]["proof_bin"]
        with pytest.raises(nzcb.NzcbError):         # a gather that fails fails the proof
            ctx.set_msm_split(world, ranks.ranges[0][1], ranks.send, lambda slot, own: b"", ranks.own_lagrange)
            ctx.prove_raw(wtns, bytes(352))
    finally:
        ranks.close()
        ctx.close()


def test_lagrange_table_ranges_add_up():
    """nzcb_msm_table_create_lagrange: ranges of the Lagrange basis computed on the GPU from a
    PTau, run with the sparse schedule, add up to the MSM over the whole basis as the
    oracle computes it (tau known: [L_k(tau)] G1 and the two blinding points)."""
    import nzcb
    from nzcb import msmsplit
    from oracle import bn254 as bn
    import random
    log_n = 6
    n = 1 << log_n
    tau = 0x7A0 + 0x6E7A6362746175
    pts = [bn.g1_mul(bn.G1_GEN, pow(tau, i, bn.R_MOD)) for i in range(n + 6)]
    w, tn = bn.FR_W[log_n], pow(tau, n, bn.R_MOD)
    inv_n = pow(n, bn.R_MOD - 2, bn.R_MOD)
    lk = [pow(w, k, bn.R_MOD) * (tn - 1) * inv_n * pow((tau - pow(w, k, bn.R_MOD)) % bn.R_MOD, bn.R_MOD - 2,
                                                          bn.R_MOD) % bn.R_MOD for k in range(n)]
    lk += [(tn - 1) % bn.R_MOD, (pow(tau, n + 1, bn.R_MOD) - tau) % bn.R_MOD]   # [tau^n]-[1], [tau^(n+1)]-[tau]
    rng = random.Random(0x1A6)
    sc = [rng.choice([0, 1, 1, bn.R_MOD - 1, rng.randrange(256), rng.randrange(bn.R_MOD)]) for _ in range(n + 2)]
    want = bn.g1_mul(bn.G1_GEN, sum(s * l for s, l in zip(sc, lk)) % bn.R_MOD)
    dp, ds = nzcb.dev_alloc(64 * (n + 6)), nzcb.dev_alloc(32 * (n + 2))
    try:
        nzcb.h2d(dp, b"".join(bn.g1_to_lem(p) for p in pts))
        nzcb.h2d(ds, b"".join(s.to_bytes(32, "little") for s in sc))
        acc = None
        for lo, hi in msmsplit.point_ranges(n + 2, 3):
            t = nzcb.MsmTable.lagrange(dp, n + 6, log_n, lo, hi)
            p = t.run(ds + 32 * lo, hi - lo, False)
            t.close()
            x, y = bn.from_le(p[:32]), bn.from_le(p[32:])
            acc = bn.g1_add(acc, None if x == 0 and y == 0 else (x, y))
        with pytest.raises(nzcb.NzcbError):
            nzcb.MsmTable.lagrange(dp, n + 1, log_n, 0, 4)      # fewer than n + 2 PTau points
        with pytest.raises(nzcb.NzcbError):
            nzcb.MsmTable.lagrange(dp, n + 6, log_n, 5, n + 3)  # past the n + 2 basis points
    finally:
        nzcb.dev_free(dp)
        nzcb.dev_free(ds)
    assert acc == want


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
