"""GPU kernel parity: field mul, NTT, MSM through the C-ABI vs the CPU oracle.

Bit-exact: every output is a unique field / affine-curve element.
"""
import os
import random

import pytest

from oracle import bn254 as bn
from oracle.bn254 import P_MOD, R_MOD

pytestmark = pytest.mark.gpu


def _lem(vals, mod):
    return b"".join(bn.to_lem(v, mod) for v in vals)


def _from_lem(data, mod):
    return [bn.from_lem(data[i:i + 32], mod) for i in range(0, len(data), 32)]


@pytest.mark.parametrize("field_q", [0, 1])
def test_field_mul(engine, field_q):
    mod = P_MOD if field_q else R_MOD
    rng = random.Random(7 + field_q)
    a = [rng.randrange(mod) for _ in range(1000)] + [0, 1, mod - 1, mod - 1]
    b = [rng.randrange(mod) for _ in range(1000)] + [mod - 1, mod - 1, mod - 1, 1]
    out = _from_lem(engine.field_mul(_lem(a, mod), _lem(b, mod), bool(field_q)), mod)
    assert out == [x * y % mod for x, y in zip(a, b)]


@pytest.mark.parametrize("log_n", [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14])
@pytest.mark.parametrize("inverse", [False, True])
def test_ntt(engine, log_n, inverse):
    """Against the oracle's FFT. 2^0..2^8 are one pass of log n stages, 2^9..2^14 a pass of 8
    and one of 1..6 (7 at 2^23, test_ntt_full_size_properties): every stage plan of the pass
    kernel (radix-8 groups of 3, radix-4 pairs, a single radix-2 stage; ntt.hip) runs, in the
    first pass and in a later one."""
    rng = random.Random(log_n * 2 + inverse)
    n = 1 << log_n
    a = [rng.randrange(R_MOD) for _ in range(n)]
    got = _from_lem(engine.ntt(_lem(a, R_MOD), log_n, inverse), R_MOD)
    want = bn.ifft(a) if inverse else bn.fft(a)
    assert got == want


@pytest.mark.parametrize("log_n", [17, 18, 20, 21, 22, 23, 24])
def test_ntt_full_size_properties(log_n):
    """The prover's NTT sizes (n = 2^21, 4n = 2^23), the top of BASELINE configs[1] (2^24)
    and the other sizes of the two-pass plan (2048-element tiles, 17 <= log n <= 22),
    size-independent properties on pseudo-random Montgomery inputs:
    iNTT(NTT(x)) = x bit-exactly; NTT(x)[0] = sum x; NTT(x)[n/2] = alternating sum;
    NTT(x)[1] and NTT(x)[n-1] against Horner at w and w^-1 (every twiddle contributes;
    at 2^21 and 2^24). All linear, so the checks run on the raw Montgomery values."""
    import nzcb
    n = 1 << log_n
    eng = nzcb.Engine(0, max_log_ntt=log_n, max_msm_points=0)
    dev = nzcb.dev_alloc(n * 32)
    try:
        eng.random_fr(dev, n, 0x4E5454 + log_n)
        data = nzcb.d2h(dev, n * 32)
        fwd = eng.ntt(data, log_n, False)
        assert eng.ntt(fwd, log_n, True) == data
    finally:
        nzcb.dev_free(dev)
        eng.close()
    x = [int.from_bytes(data[i:i + 32], "little") for i in range(0, 32 * n, 32)]
    y = [int.from_bytes(fwd[i:i + 32], "little") for i in (0, 32, 32 * (n // 2), 32 * (n - 1))]
    assert y[0] == sum(x) % R_MOD
    assert y[2] == (sum(x[0::2]) - sum(x[1::2])) % R_MOD
    if log_n != 23:
        w = bn.FR_W[log_n]
        assert y[1] == bn.eval_pol(x, w)
        assert y[3] == bn.eval_pol(x, bn.fr_inv(w))


def _affine(out):
    x = bn.from_le(out[:32])
    y = bn.from_le(out[32:])
    return None if x == 0 and y == 0 else (x, y)


def _bases(n, seed):
    rng = random.Random(seed)
    pts = []
    p = bn.g1_mul(bn.G1_GEN, rng.randrange(1, R_MOD))
    step = bn.g1_mul(bn.G1_GEN, rng.randrange(1, R_MOD))
    for _ in range(n):
        pts.append(p)
        p = bn.g1_add(p, step)
    return pts


@pytest.mark.parametrize("n,kind", [(1, "rand"), (7, "rand"), (100, "rand"), (1000, "rand"), (3000, "rand"),
                                    (300, "zeros"), (300, "ones"), (300, "equal"), (300, "rminus1"),
                                    (300, "small"), (300, "mixed")])
def test_msm(engine, n, kind):
    rng = random.Random(n + len(kind))
    pts = _bases(n, n)
    if kind == "rand":
        sc = [rng.randrange(R_MOD) for _ in range(n)]
    elif kind == "zeros":
        sc = [0] * n
    elif kind == "ones":
        sc = [1] * n
    elif kind == "equal":
        v = rng.randrange(R_MOD)
        sc = [v] * n
    elif kind == "rminus1":
        sc = [R_MOD - 1] * n
    elif kind == "small":
        sc = [rng.randrange(1 << 20) for _ in range(n)]
    else:
        sc = [rng.choice([0, 1, R_MOD - 1, rng.randrange(R_MOD)]) for _ in range(n)]
    bases = b"".join(bn.g1_to_lem(p) for p in pts)
    want = bn.msm(pts, sc)
    got = _affine(engine.msm(bases, b"".join(bn.to_le(s) for s in sc), False))
    assert got == want
    got_m = _affine(engine.msm(bases, _lem(sc, R_MOD), True))
    assert got_m == want


def test_msm_duplicate_and_negated_points(engine):
    g = bn.g1_mul(bn.G1_GEN, 12345)
    pts = [g, g, bn.g1_neg(g), g, None, g]
    sc = [5, 5, 5, 7, 9, R_MOD - 5]
    want = bn.msm(pts, sc)
    bases = b"".join(bn.g1_to_lem(p) for p in pts)
    got = _affine(engine.msm(bases, b"".join(bn.to_le(s) for s in sc), False))
    assert got == want


def _msm_fixed(engine, pts, sc, n_table=None, mont=False, window=0, sparse=False):
    """Fixed-base schedule (shifted-base table, one 2^19-bucket set) via device buffers;
    window / sparse: another table window, the Lagrange table's sparse schedule."""
    import nzcb
    n = len(sc)
    n_table = n_table or n
    bases = b"".join(bn.g1_to_lem(p) for p in pts[:n_table])
    scal = _lem(sc, R_MOD) if mont else b"".join(bn.to_le(s) for s in sc)
    db, ds = nzcb.dev_alloc(len(bases)), nzcb.dev_alloc(max(len(scal), 32))
    try:
        nzcb.h2d(db, bases)
        if scal:
            nzcb.h2d(ds, scal)
        return _affine(engine.msm_fixed_dev(db, n_table, ds, n, mont, window=window, sparse=sparse))
    finally:
        nzcb.dev_free(db)
        nzcb.dev_free(ds)


def _flip_kinds(kind, n, rng):
    """Scalars for the signed-scalar bucketing (msm.hip scalar_min_form: min(s, r - s) with
    the base negated): "half" sits on the (r - 1) / 2 boundary on both sides, "negsmall" is
    the A, B, C regime of small negatives r - k next to small positives and their sums with
    equal bases' opposite signs in one bucket. None for any other kind."""
    h = (R_MOD - 1) // 2
    if kind == "half":
        return [rng.choice([h, h + 1, h - 1, h + 2, R_MOD - 1, 1, R_MOD - (1 << 16), (1 << 16) + 1,
                            rng.randrange(h - 1000, h + 1000)]) for _ in range(n)]
    if kind == "negsmall":
        return [rng.choice([0, 1, R_MOD - 1, R_MOD - 2, 2, rng.randrange(256), R_MOD - rng.randrange(1, 256),
                            R_MOD - rng.randrange(1, 1 << 17), rng.randrange(1 << 17),
                            R_MOD - rng.randrange(1, 1 << 40)]) for _ in range(n)]
    return None


@pytest.mark.parametrize("n,kind", [(1, "rand"), (100, "rand"), (2000, "rand"), (300, "zeros"), (300, "ones"),
                                    (300, "equal"), (300, "rminus1"), (300, "mixed"), (300, "top"),
                                    (3000, "witness"), (600, "half"), (2000, "negsmall")])
def test_msm_fixed_base(engine, n, kind):
    rng = random.Random(1000 + n + len(kind))
    pts = _bases(n + 5, n + 1)
    if kind == "rand":
        sc = [rng.randrange(R_MOD) for _ in range(n)]
    elif kind == "zeros":
        sc = [0] * n
    elif kind == "ones":
        sc = [1] * n
    elif kind == "equal":
        sc = [rng.randrange(R_MOD)] * n
    elif kind == "rminus1":
        sc = [R_MOD - 1] * n
    elif kind == "witness":  # gate values as the Lagrange-basis commitments see them: mostly zero
        # digits (0, 1, -1, bytes, 17/34-bit sums), a few full-size inverses
        sc = [rng.choice([0, 0, 1, 1, R_MOD - 1, rng.randrange(256), rng.randrange(1 << 17),
                          rng.randrange(1 << 34), rng.randrange(R_MOD)]) for _ in range(n)]
    elif kind == "top":  # digits at the top window edge: 2^240.., 2^253, half-window carries
        sc = [rng.choice([1 << 253, (1 << 240) - 1, (1 << 239) * 3, (1 << 19) * 5, R_MOD - (1 << 19)])
              for _ in range(n)]
    else:
        sc = _flip_kinds(kind, n, rng)
    if sc is None:
        sc = [rng.choice([0, 1, R_MOD - 1, rng.randrange(R_MOD)]) for _ in range(n)]
    want = bn.msm(pts[:n], sc)
    # table built over more bases than the MSM uses (as the prover's n+6 PTau table)
    assert _msm_fixed(engine, pts, sc, n_table=n + 5) == want
    assert _msm_fixed(engine, pts, sc, n_table=n + 5, mont=True) == want


@pytest.mark.parametrize("n,kind", [(1, "rand"), (300, "rand"), (300, "zeros"), (3000, "ones"), (1500, "equal"),
                                    (300, "rminus1"), (300, "top"), (3000, "witness"), (5000, "equal"),
                                    (2000, "mixed"), (16, "equal"), (600, "half"), (3000, "negsmall")])
def test_msm_sparse_schedule(engine, n, kind):
    """The Lagrange table's schedule (round 6, msm.hip dyn_chunk): window 17, the accumulation
    chunk derived on the device from the entry count (8 entries here), runs of more than four
    carries through the log-depth piece and bucket trees. "ones" and "equal" put thousands of
    entries into single buckets (1 to 3 pieces per bucket), "witness" is the A, B, C regime."""
    rng = random.Random(4000 + n + len(kind))
    pts = _bases(n + 2, 2 * n + 3)
    if kind == "rand":
        sc = [rng.randrange(R_MOD) for _ in range(n)]
    elif kind == "zeros":
        sc = [0] * n
    elif kind == "ones":
        sc = [1] * n
    elif kind == "equal":
        sc = [rng.randrange(R_MOD)] * n
    elif kind == "rminus1":
        sc = [R_MOD - 1] * n
    elif kind == "top":
        sc = [rng.choice([1 << 253, (1 << 240) - 1, (1 << 16) * 5, R_MOD - (1 << 16)]) for _ in range(n)]
    elif kind == "witness":
        sc = [rng.choice([0, 0, 1, 1, 1, R_MOD - 1, rng.randrange(256), rng.randrange(1 << 17),
                          rng.randrange(R_MOD)]) for _ in range(n)]
    else:
        sc = _flip_kinds(kind, n, rng)
    if sc is None:
        sc = [rng.choice([0, 1, 2, R_MOD - 1, rng.randrange(R_MOD)]) for _ in range(n)]
    want = bn.msm(pts[:n], sc)
    assert _msm_fixed(engine, pts, sc, n_table=n + 2, window=17, sparse=True) == want
    assert _msm_fixed(engine, pts, sc, n_table=n + 2, mont=True, window=17, sparse=True) == want


@pytest.mark.parametrize("n,kinds", [(1, ("rand", "ones", "zeros")), (300, ("witness", "equal", "rand")),
                                     (3000, ("ones", "witness", "mixed")), (1500, ("equal", "equal", "ones")),
                                     (700, ("zeros", "zeros", "witness")), (2000, ("witness", "rand")),
                                     (1200, ("negsmall", "half", "negsmall"))])
def test_msm_sets_schedule(engine, n, kinds):
    """msm_enqueue_sets (round 6: the prover's A, B, C in one schedule over the Lagrange table):
    each set's result equals its own MSM (oracle), for sets whose buckets collide in index
    (equal scalars in two sets), empty sets, huge single buckets (ones, equal) and the
    witness-like regime; Montgomery and normal-form scalars."""
    import nzcb
    rng = random.Random(5000 + n + len(kinds))
    pts = _bases(n + 2, 3 * n + 11)

    def scal(kind):
        if kind == "rand":
            return [rng.randrange(R_MOD) for _ in range(n)]
        if kind == "zeros":
            return [0] * n
        if kind == "ones":
            return [1] * n
        if kind == "equal":
            return [rng.randrange(R_MOD)] * n
        if kind == "witness":
            return [rng.choice([0, 0, 1, 1, 1, R_MOD - 1, rng.randrange(256), rng.randrange(1 << 17),
                                rng.randrange(R_MOD)]) for _ in range(n)]
        if kind in ("half", "negsmall"):
            return _flip_kinds(kind, n, rng)
        return [rng.choice([0, 1, 2, R_MOD - 1, rng.randrange(R_MOD)]) for _ in range(n)]

    sets = [scal(k) for k in kinds]
    if kinds == ("equal", "equal", "ones"):
        sets[1] = list(sets[0])   # the same bucket in two sets
    want = [bn.msm(pts[:n], sc) for sc in sets]
    bases = b"".join(bn.g1_to_lem(p) for p in pts)
    db = nzcb.dev_alloc(len(bases))
    ds = [nzcb.dev_alloc(32 * n) for _ in sets]
    try:
        nzcb.h2d(db, bases)
        for mont in (False, True):
            for d, sc in zip(ds, sets):
                nzcb.h2d(d, _lem(sc, R_MOD) if mont else b"".join(bn.to_le(x) for x in sc))
            got = [_affine(r) for r in engine.msm_sets_dev(db, n + 2, ds, n, mont)]
            assert got == want, (mont, [g == w for g, w in zip(got, want)])
    finally:
        nzcb.dev_free(db)
        for d in ds:
            nzcb.dev_free(d)


def test_msm_fixed_base_infinity_bases(engine):
    g = bn.g1_mul(bn.G1_GEN, 777)
    pts = [g, None, bn.g1_neg(g), g, None, g]
    sc = [5, 6, 5, 7, 9, R_MOD - 5]
    assert _msm_fixed(engine, pts, sc) == bn.msm(pts, sc)


@pytest.mark.parametrize("fixed", [False, True])
def test_msm_long_carry_runs(engine, fixed):
    """Equal scalars put every window's entries in one bucket: thousands of accumulation
    chunks end in carries of one bucket (the finalize kernel's workgroup path)."""
    n = 5000
    rng = random.Random(77)
    pts = _bases(n, 4242)
    v = rng.randrange(R_MOD)
    sc = [v] * n
    acc = None
    for p in pts:
        acc = bn.g1_add(acc, p)
    want = bn.g1_mul(acc, v)
    if fixed:
        assert _msm_fixed(engine, pts, sc) == want
    else:
        bases = b"".join(bn.g1_to_lem(p) for p in pts)
        got = _affine(engine.msm(bases, b"".join(bn.to_le(s) for s in sc), False))
        assert got == want


@pytest.mark.parametrize("kind", ["rand", "equal", "mixed", "small"])
def test_msm_fixed_base_digit_patterns(engine, kind):
    """Bucket runs of every shape: equal scalars put a window's entries in one bucket (runs
    spanning many accumulation chunks: the finalize's large list), "small" scalars leave
    most windows zero (no entries), "mixed" has 0, 1, 2, r - 1 and random scalars."""
    n = 1500
    rng = random.Random(31 + len(kind))
    pts = _bases(n, 900 + len(kind))
    if kind == "rand":
        sc = [rng.randrange(R_MOD) for _ in range(n)]
    elif kind == "equal":
        sc = [rng.randrange(R_MOD)] * n
    elif kind == "small":
        sc = [rng.randrange(1 << 24) for _ in range(n)]
    else:
        sc = [rng.choice([0, 1, 2, R_MOD - 1, rng.randrange(R_MOD)]) for _ in range(n)]
    assert _msm_fixed(engine, pts, sc) == bn.msm(pts, sc)


def test_msm_fixed_base_doublings_and_cancellations(engine):
    """Equal points in one bucket (the accumulation doubles), a point and its negation (the
    bucket sum is infinity), infinity bases, and equal partial sums meeting in the finalize
    and the window sum's trees."""
    g = bn.g1_mul(bn.G1_GEN, 4321)
    h = bn.g1_mul(bn.G1_GEN, 99)
    pts = [g, g, bn.g1_neg(g), g, None, g, h, h, bn.g1_neg(h), None, g, g, g, g, h, bn.g1_neg(g)]
    sc = [5, 5, 5, 5, 5, R_MOD - 5, 5, 5, 5, 7, 5, 5, 5, 5, R_MOD - 5, 5]
    assert _msm_fixed(engine, pts, sc) == bn.msm(pts, sc)


def test_msm_large_chunks_schedules_agree_and_split_linearly():
    """2^22 points (about 63-67 M bucket entries): the accumulation chunk doubles past
    2^25 entries (msm.hip chunk_for). The generic schedule (c = 16 windows) and the
    fixed-base table schedule (c = 17, 29-bit radix) are independent code paths and
    must agree, and MSM(P, s) = MSM(P[:h], s[:h]) + MSM(P[h:], s[h:]) (size-independent)."""
    import nzcb
    n, h = 1 << 22, 1 << 21
    eng = nzcb.Engine(0, max_log_ntt=-1, max_msm_points=n + 8)
    sc, bases = nzcb.dev_alloc(n * 32), nzcb.dev_alloc(n * 64)
    try:
        eng.random_fr(sc, n, 0x6E7A6362)
        eng.fixed_base(sc, n, bases)          # bases_i = [s_i] G1, affine LEM
        eng.random_fr(sc, n, 0x5EED)          # fresh scalars (Montgomery)
        generic = _affine(eng.msm_dev(bases, sc, n, True))
        fixed = _affine(eng.msm_fixed_dev(bases, n, sc, n, True))
        lo = _affine(eng.msm_fixed_dev(bases, h, sc, h, True))
        hi = _affine(eng.msm_fixed_dev(bases + h * 64, n - h, sc + h * 32, n - h, True))
    finally:
        nzcb.dev_free(sc)
        nzcb.dev_free(bases)
        eng.close()
    assert generic is not None and generic == fixed
    assert bn.g1_add(lo, hi) == fixed


@pytest.mark.parametrize("log_n", [1, 3, 6, 9])
def test_lagrange_basis_vs_oracle(engine, log_n):
    """csrc/lagrange.hip (an elliptic-curve iNTT of PTau): [L_k(tau)] for every k, then
    [tau^n] - [1] and [tau^(n+1)] - [tau], against the oracle's scalars times G1 with the
    trapdoor tau known."""
    import nzcb
    n = 1 << log_n
    tau = 0x6E7A6362746175 + log_n
    pts = [bn.g1_mul(bn.G1_GEN, pow(tau, i, R_MOD)) for i in range(n + 6)]
    w = bn.FR_W[log_n]
    tn = pow(tau, n, R_MOD)
    inv_n = pow(n, R_MOD - 2, R_MOD)
    want = []
    for k in range(n):
        wk = pow(w, k, R_MOD)
        # L_k(tau) = w^k (tau^n - 1) / (n (tau - w^k))
        lk = wk * (tn - 1) * inv_n * pow((tau - wk) % R_MOD, R_MOD - 2, R_MOD) % R_MOD
        want.append(bn.g1_mul(bn.G1_GEN, lk))
    want.append(bn.g1_add(pts[n], bn.g1_neg(pts[0])))
    want.append(bn.g1_add(pts[n + 1], bn.g1_neg(pts[1])))
    dp, do = nzcb.dev_alloc(64 * (n + 6)), nzcb.dev_alloc(64 * (n + 2))
    try:
        nzcb.h2d(dp, b"".join(bn.g1_to_lem(p) for p in pts))
        engine.lagrange_basis(dp, n + 6, log_n, do)
        out = nzcb.d2h(do, 64 * (n + 2))
    finally:
        nzcb.dev_free(dp)
        nzcb.dev_free(do)
    got = [bn.g1_from_lem(out[64 * k:64 * k + 64]) for k in range(n + 2)]
    assert got == want



@pytest.mark.parametrize("window", ["16", "17", "19"])
def test_msm_fixed_base_other_windows(window):
    """The fixed-base tests above under the windows NZCB_FB_WINDOW selects besides the default
    c = 20 (c = 16, 17: the LDS tile kernel of the window sum; c = 19: 2^18 buckets, strips; a fresh
    process, the switch is read once)."""
    import subprocess
    import sys
    env = dict(os.environ, NZCB_FB_WINDOW=window)
    p = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", "-m", "gpu",
                        os.path.abspath(__file__), "-k", "fixed_base and not other_windows"],
                       capture_output=True, text=True, timeout=110, env=env)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-2000:]


# --- csrc/f29.h products as the device compiles them -------------------------
_M29 = (1 << 29) - 1
_RINV261 = {m: pow(2, -261, m) for m in (P_MOD, R_MOD)}


def _l29(x):
    return [(x >> (29 * i)) & _M29 for i in range(9)]


def _v29(ws):
    return sum(v << (29 * i) for i, v in enumerate(ws))


def _wide29(x, rng):
    """x's limbs with random borrows moved down (limbs above 2^29, below 2^30.7): the
    unnormalized inputs the NTT passes hand to the Shoup product."""
    xl = _l29(x)
    for i in range(8, 0, -1):
        if xl[i] and rng.random() < 0.5:
            b = rng.randrange(0, min(xl[i], 3) + 1)
            xl[i] -= b
            xl[i - 1] += b << 29
    return xl if max(xl) < int(2 ** 30.7) else _l29(x)


def test_f29_device_products_exact():
    """Every generated column-asm product of csrc/f29_cols.h on the GPU (nzcb_debug_f29)
    against exact integers, at and near the bounds the kernels rely on: the Shoup twiddle
    product (single and paired; x < 99 r < 2^261 with limbs up to 2^30.7, result = x w mod r
    and < 3 r), the Montgomery products mod q and mod r (inputs < 2 p, result < 2 p), the
    paired squaring and the two-product sum (inputs < 4 q, result congruent and < 4 q).
    Output limbs are normalized (< 2^29) except the top one."""
    import nzcb
    rng = random.Random(0xF29C)
    N = 2000
    R, Q = R_MOD, P_MOD
    edge = lambda m: [0, 1, m - 1, 2 * m - 1]

    # op 1 / 2: Shoup
    xs = [99 * R - 1, R - 1, 0] + [rng.randrange(99 * R) for _ in range(N)]
    ws = [R - 1, R - 1, 5] + [rng.randrange(R) for _ in range(N)]
    words, items = [], []
    for x, w in zip(xs, ws):
        xl = _wide29(x, rng)
        items.append((x, w))
        words += xl + _l29(w) + _l29((w << 261) // R)
    out = nzcb.f29_check(1, words)
    for i, (x, w) in enumerate(items):
        g = out[9 * i:9 * i + 9]
        assert max(g[:8]) <= _M29 and _v29(g) % R == x * w % R and _v29(g) < 3 * R, i
    pairs = list(zip(items[0::2], items[1::2]))
    words = []
    for (x, w), (y, v) in pairs:
        words += _wide29(x, rng) + _l29(w) + _l29((w << 261) // R) + _wide29(y, rng) + _l29(v) + _l29((v << 261) // R)
    out = nzcb.f29_check(2, words)
    for i, ((x, w), (y, v)) in enumerate(pairs):
        g1, g2 = out[18 * i:18 * i + 9], out[18 * i + 9:18 * i + 18]
        assert _v29(g1) % R == x * w % R and _v29(g1) < 3 * R, i
        assert _v29(g2) % R == y * v % R and _v29(g2) < 3 * R, i

    # op 3: mul29<Fq29>, op 4: mul29x2<Fr29>
    for op, m in ((3, Q), (4, R)):
        a = edge(m) + [rng.randrange(2 * m) for _ in range(N)]
        b = edge(m)[::-1] + [rng.randrange(2 * m) for _ in range(N)]
        k = len(a) // 2 * 2
        words = []
        if op == 3:
            for x, y in zip(a, b):
                words += _l29(x) + _l29(y)
        else:
            for j in range(0, k, 2):
                words += _l29(a[j]) + _l29(b[j]) + _l29(a[j + 1]) + _l29(b[j + 1])
        out = nzcb.f29_check(op, words)
        cnt = len(a) if op == 3 else k
        for i in range(cnt):
            g = out[9 * i:9 * i + 9]
            assert max(g[:8]) <= _M29, (op, i)
            assert _v29(g) % m == a[i] * b[i] * _RINV261[m] % m and _v29(g) < 2 * m, (op, i)

    # op 5: sqr29x2 (mod q), op 6: mul2sum29 (mod q), inputs < 4 q
    a = [4 * Q - 1, 0, Q] + [rng.randrange(4 * Q) for _ in range(N)]
    c = [4 * Q - 1, 1, Q - 1] + [rng.randrange(4 * Q) for _ in range(N)]
    words = []
    for x, y in zip(a, c):
        words += _l29(x) + _l29(y)
    out = nzcb.f29_check(5, words)
    for i, (x, y) in enumerate(zip(a, c)):
        g1, g2 = out[18 * i:18 * i + 9], out[18 * i + 9:18 * i + 18]
        assert _v29(g1) % Q == x * x * _RINV261[Q] % Q and _v29(g1) < 4 * Q, i
        assert _v29(g2) % Q == y * y * _RINV261[Q] % Q and _v29(g2) < 4 * Q, i
    b = [rng.randrange(4 * Q) for _ in a]
    d = [rng.randrange(4 * Q) for _ in a]
    words = []
    for w4 in zip(a, b, c, d):
        for v in w4:
            words += _l29(v)
    out = nzcb.f29_check(6, words)
    for i, (x, y, z, t) in enumerate(zip(a, b, c, d)):
        g = out[9 * i:9 * i + 9]
        assert _v29(g) % Q == (x * y + z * t) * _RINV261[Q] % Q and _v29(g) < 4 * Q, i
