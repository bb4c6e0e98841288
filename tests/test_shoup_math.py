"""The NTT's twiddle product (csrc/f29.h mul_shoup, round 5) restated limb for limb in
exact integers: the quotient from columns 7..16 of x * ws only, the result from the low
columns of x * w + q * (2^261 - r), for inputs at the bounds the NTT passes hold (values
< 99 r with limbs up to 2^30.7, ntt.hip). Every column stays below 2^64, the result is
x * w mod r up to a multiple of r and below 3r, and the twiddle table's ws from the
Montgomery-261 form (ntt.hip ntt_tw29_kernel) equals floor(w 2^261 / r)."""
import random

from oracle.bn254 import R_MOD as R

M = (1 << 29) - 1
RP = (1 << 261) - R
NINV = (-pow(R, -1, 1 << 261)) % (1 << 261)


def limbs(x):
    return [(x >> (29 * i)) & M for i in range(9)]


def val(l):
    return sum(v << (29 * i) for i, v in enumerate(l))


def mul_shoup(x, w, ws):
    rp = limbs(RP)
    acc, q = 0, [0] * 9
    for c in range(7, 17):
        for j in range(max(0, c - 8), min(c, 8) + 1):
            acc += x[j] * ws[c - j]
        assert acc < 1 << 64
        if c >= 9:
            q[c - 9] = acc & M
        acc >>= 29
    q[8] = acc
    acc, out = 0, [0] * 9
    for c in range(9):
        for j in range(c + 1):
            acc += x[j] * w[c - j] + q[j] * rp[c - j]
        assert acc < 1 << 64
        out[c] = acc & M
        acc >>= 29
    return out


def _wide(X, rng):
    """X as 9 limbs with some value moved into lower limbs (limbs up to 2^30.7)."""
    xl = limbs(X)
    for i in range(8, 0, -1):
        if xl[i] and rng.random() < 0.5:
            b = rng.randrange(0, min(xl[i], 3) + 1)
            xl[i] -= b
            xl[i - 1] += b << 29
    if max(xl) >= int(2 ** 30.7):
        xl = limbs(X)
    assert val(xl) == X
    return xl


def test_shoup_product_bounds_and_value():
    rng = random.Random(0x5400)
    edge_w = [0, 1, R - 1, (R - 1) // 2, 1 << 253]
    edge_x = [0, 1, R - 1, 99 * R - 1, (1 << 261) - 1, 3 * R]
    cases = [(w, x) for w in edge_w for x in edge_x]
    cases += [(rng.randrange(R), rng.randrange(99 * R)) for _ in range(3000)]
    for W, X in cases:
        m = (W << 261) % R                       # the twiddle's Montgomery-261 form
        ws = (m * NINV) % (1 << 261)             # ntt_tw29_kernel's ws
        assert ws == (W << 261) // R
        out = mul_shoup(_wide(X, rng), limbs(W), limbs(ws))
        v = val(out)
        assert all(l <= M for l in out)
        assert v % R == (X * W) % R and v < 3 * R


def test_ntt_value_bound():
    """After L <= 24 butterfly stages from inputs < 2.4 r, each adding at most 4r (a + 4r - t,
    t < 3r), values stay below 99 r < 2^260.3: every product input < 2^261."""
    bound = 2.4 + 4 * 24
    assert bound < 99 and 99 * R < 2 ** 260.3
