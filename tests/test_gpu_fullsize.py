"""configs[2] and the top of configs[1] at full size.

* The bench's exact workload (bench.py: n = 2^21, nPublic = 3, 2970 inputs, seeded
  synthetic circuit with free public wires, live-shaped passes) proved once through
  nzcb_prove_device and as a 3-lane nzcb_prove_batch (fullProve: nzcp witness kernel ->
  witness[1..3] in HBM -> proof). Every proof byte and public signal is compared with the
  C port (oracle/c/nzcb_ref.c) on the same zkey, witness and fixed blinding; the nzcp
  outputs with the CPU restatement (oracle/nzcp_circuit.py, pinned by the reference's KATs).
  At 2^21 the fixed-base MSM runs 31.5 M bucket entries per launch, a chunk/carry regime
  the small parity tests never reach.
* A 2^24-point MSM (configs[1] top): the generic and fixed-base schedules agree, and the
  fixed-base MSM splits linearly over two point ranges.

Prover parity against snarkjs itself stays unpinned: the C port is the
builder's restatement, an implementation independent of the HIP kernels.
"""
import ctypes

import pytest

import bench
import nzcp_cases as C
from oracle import nzcp_circuit as nz
from oracle import synth

pytestmark = pytest.mark.gpu


def _affine(out):
    from oracle import bn254 as bn
    x, y = bn.from_le(out[:32]), bn.from_le(out[32:])
    return None if x == 0 and y == 0 else (x, y)


@pytest.mark.timeout(900)
def test_nzcp_live_2p21_bit_exact_vs_c_port():
    import nzcb
    from oracle import cbind
    raw = nzcb.synth_setup_raw(21, 3, bench.NZCP_INPUTS, bench.SEED, 0, bench.TAU, free_public=True)
    try:
        ctx = nzcb.ProverContext(None, _raw=(raw[0], raw[1]))
        wtns = ctypes.string_at(raw[2], raw[3])
        nwit = (len(wtns) - 76) // 32
        assert ctx.domain_size == 1 << 21 and ctx.n_public == 3
        base = wtns[76:76 + 32 * nwit]
        prover = nzcb.NzcpProver(ctx, base)
        idx = [0, 1, 2]
        passes = [C.case(f"live{i}", nz.LIVE_PARAMS, C.live_tbs(), data=bench.pass_data(i)) for i in idx]
        inputs = bench.pass_inputs(idx)
        assert inputs == b"".join(C.case_input_bytes(c) for c in passes)
        bl = b"".join(x.to_bytes(32, "little") for x in synth.fixed_blindings())
        bl2 = bench.blinding_for(7)
        try:
            ctx.set_lanes(3)
            res, recs = prover.full_prove(inputs, [bl, bl, bl2])
            # the same pass-0 witness straight through nzcb_prove_device
            (w0,) = prover.witness_buffers(1)[:1]
            dev_proof, dev_pub = ctx.prove_device_raw(w0, nwit, bl)
        finally:
            prover.close()
        exp_out = [[int(v) for v in C.oracle_record(c)["out"]] for c in passes]
        for (proof, pub), r, e in zip(res, recs, exp_out):
            assert r["status"] == 0 and r["out"] == e
            assert [int.from_bytes(pub[32 * k:32 * k + 32], "little") for k in range(3)] == e
        # C port on the witnesses of passes 0 and 1 (publics replaced by the restatement's)
        refs = []
        for e in exp_out[:2]:
            w = bytearray(wtns)
            for k in range(3):
                w[76 + 32 * (1 + k):76 + 32 * (2 + k)] = e[k].to_bytes(32, "little")
            wb = bytes(w)
            refs.append(cbind.prove((raw[0], raw[1]), wb, bl, npub=3)[:2])
        assert dev_proof == refs[0][0] and dev_pub == refs[0][1][:96]
        assert res[0][0] == refs[0][0] and res[0][1] == refs[0][1][:96]
        assert res[1][0] == refs[1][0] and res[1][1] == refs[1][1][:96]
        # third lane: other blinding, same statement as pass 2 -> a different valid proof
        assert res[2][0] not in (refs[0][0], refs[1][0])
        assert all(nzcb.verify(ctx.vk, p, q) for p, q in res)
        # round 4's overrun (k_t_combine writing t[3n..4n) into the 3n + 6
        # quotient buffer) surfaced two kernels later as an illegal access in this test.
        # Every buffer of the context (proving key, 3 lanes' working sets, MSM and NTT
        # scratch) carries guard words: all intact after the 3-lane batch and the single proof
        checked = nzcb.guard_check(0)
        assert checked >= 3 * 40
        ctx.close()
    finally:
        nzcb.free_raw(raw)


@pytest.mark.timeout(600)
def test_msm_2p24_vs_c_port_and_split_linearly():
    """2^24 points, the top of BASELINE configs[1]: 252 M fixed-base bucket entries. Both GPU
    schedules (generic and fixed-base) equal the C port's MSM (oracle/c/nzcb_ref.c, an
    independent Pippenger on the host) on the same bases and scalars, and the fixed-base
    schedule splits linearly over point ranges."""
    import nzcb
    from oracle import bn254 as bn
    from oracle import cbind
    n, h = 1 << 24, (1 << 23) + 12345
    eng = nzcb.Engine(0, max_log_ntt=-1, max_msm_points=n + 8)
    sc, bases = nzcb.dev_alloc(n * 32), nzcb.dev_alloc(n * 64)
    try:
        eng.random_fr(sc, n, 0x32343234)
        eng.fixed_base(sc, n, bases)
        eng.random_fr(sc, n, 0x5EED24)
        generic = _affine(eng.msm_dev(bases, sc, n, True))
        fixed = _affine(eng.msm_fixed_dev(bases, n, sc, n, True))
        lo = _affine(eng.msm_fixed_dev(bases, h, sc, h, True))
        hi = _affine(eng.msm_fixed_dev(bases + h * 64, n - h, sc + h * 32, n - h, True))
        host_bases, host_scalars = nzcb.d2h(bases, n * 64), nzcb.d2h(sc, n * 32)
    finally:
        nzcb.dev_free(sc)
        nzcb.dev_free(bases)
        eng.close()
    ref = _affine(cbind.msm(host_bases, host_scalars))     # LEM bases, Montgomery scalars
    assert ref is not None
    assert generic == ref and fixed == ref
    assert bn.g1_add(lo, hi) == fixed


@pytest.mark.timeout(600)
def test_msm_2p21_witness_scalars_schedules_agree():
    """The Lagrange-basis commitments' regime at full size: 2^21 + 2 scalars shaped like
    nzcp_live gate values (mostly 0, 1, -1, bytes and short sums, ~5 % full-size), so most
    digits are zero and the bucketing drops them, and bucket 0 (|digit| = 1) holds ~40 %
    of the entries (long carry runs through the finalize's workgroup path). The fixed-base
    schedule equals the generic one, which keeps every digit, and splits linearly; the sparse
    schedule the prover uses for these scalars (round 6) gives the same point."""
    import random
    import numpy as np
    import nzcb
    from oracle import bn254 as bn
    n, h = (1 << 21) + 2, (1 << 20) + 777
    rng = random.Random(0x6E7A)
    r = bn.R_MOD
    kinds = rng.choices(range(7), weights=[35, 30, 10, 10, 8, 2, 5], k=n)
    vals = [0 if k == 0 else 1 if k == 1 else r - 1 if k == 2 else rng.randrange(256) if k == 3 else
            rng.randrange(1 << 17) if k == 4 else rng.randrange(1 << 40) if k == 5 else rng.randrange(r)
            for k in kinds]
    raw = b"".join(v.to_bytes(32, "little") for v in vals)
    assert np.frombuffer(raw, dtype=np.uint8).size == 32 * n
    eng = nzcb.Engine(0, max_log_ntt=-1, max_msm_points=n + 8)
    sc, bases = nzcb.dev_alloc(n * 32), nzcb.dev_alloc(n * 64)
    try:
        eng.random_fr(sc, n, 0x1A6A)
        eng.fixed_base(sc, n, bases)
        nzcb.h2d(sc, raw)                       # normal-form scalars
        generic = _affine(eng.msm_dev(bases, sc, n, False))
        fixed = _affine(eng.msm_fixed_dev(bases, n, sc, n, False))
        lo = _affine(eng.msm_fixed_dev(bases, h, sc, h, False))
        hi = _affine(eng.msm_fixed_dev(bases + h * 64, n - h, sc + h * 32, n - h, False))
        # the Lagrange table's schedule (window 17, device-derived chunk, carry trees)
        sparse = _affine(eng.msm_fixed_dev(bases, n, sc, n, False, window=17, sparse=True))
        slo = _affine(eng.msm_fixed_dev(bases, h, sc, h, False, window=17, sparse=True))
        # and the three-set schedule (the prover's A, B, C in one MSM): the same scalars as set 0
        # and set 2, their halves' order reversed in set 1 (other buckets, same sizes)
        sc2 = nzcb.dev_alloc(n * 32)
        try:
            nzcb.h2d(sc2, raw[32 * h:] + raw[:32 * h])
            s3 = [_affine(r) for r in eng.msm_sets_dev(bases, n, [sc, sc2, sc], n, False)]
            rot = _affine(eng.msm_fixed_dev(bases, n, sc2, n, False, window=17, sparse=True))
        finally:
            nzcb.dev_free(sc2)
    finally:
        nzcb.dev_free(sc)
        nzcb.dev_free(bases)
        eng.close()
    assert generic is not None and generic == fixed
    assert bn.g1_add(lo, hi) == fixed
    assert sparse == fixed
    assert bn.g1_add(slo, hi) == fixed
    assert s3[0] == fixed and s3[2] == fixed and s3[1] == rot
