"""BN254 (alt_bn128 / "bn128") arithmetic for the CPU oracle.

TEST INFRASTRUCTURE ONLY. This package is the checker for the HIP prover in
``nzcb-circom_amd/``; only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it. Parity status: **parity
unpinned against snarkjs** (snarkjs / ffjavascript / wasmcurves are [EXT] and
absent); the primitives below are pinned by the published
BN254 constants quoted in SURVEY.md §8 (r, p, w[21], w[23], w[28]) and by
curve-equation / group-order checks in ``tests/test_oracle.py``.

Restates the field/curve layer that the reference reaches through
``snarkjs@0.4.12 -> ffjavascript@0.2.48 -> wasmcurves@0.1.0``
(``/root/reference/yarn.lock:7279-7292, 3905-3913, 8173-8179``;
SURVEY.md §8a row a13). Elements are plain Python ints in *normal* form; the
Montgomery ("LEM") representation only appears at the byte boundary
(``to_lem`` / ``from_lem``), exactly where the zkey format uses it
(SURVEY.md §8 "zkey data is in Montgomery form").
"""
from __future__ import annotations

R_MOD = 21888242871839275222246405745257275088548364400416034343698204186575808495617
P_MOD = 21888242871839275222246405745257275088696311157297823662689037894645226208583
MONT_R = 1 << 256

# ---------------------------------------------------------------------------
# Fr roots of unity, ffjavascript convention: nqr = 5, s = 28,
# w[s] = nqr^t with r-1 = 2^s * t, w[k-1] = w[k]^2  (SURVEY.md §8 constants).
# ---------------------------------------------------------------------------
FR_S = 28
_T = (R_MOD - 1) >> FR_S
FR_NQR = 5
FR_W = [0] * (FR_S + 1)
FR_W[FR_S] = pow(FR_NQR, _T, R_MOD)
for _k in range(FR_S, 0, -1):
    FR_W[_k - 1] = FR_W[_k] * FR_W[_k] % R_MOD


def fr_inv(a: int) -> int:
    if a % R_MOD == 0:
        raise ZeroDivisionError("Fr inverse of zero")
    return pow(a, R_MOD - 2, R_MOD)


def fq_inv(a: int) -> int:
    if a % P_MOD == 0:
        raise ZeroDivisionError("Fq inverse of zero")
    return pow(a, P_MOD - 2, P_MOD)


def batch_inverse(vals, mod=R_MOD):
    """Montgomery's trick (ffjavascript ``Fr.batchInverse``); zeros map to 0."""
    n = len(vals)
    pref = [1] * (n + 1)
    for i, v in enumerate(vals):
        pref[i + 1] = pref[i] * (v if v else 1) % mod
    inv = pow(pref[n], mod - 2, mod)
    out = [0] * n
    for i in range(n - 1, -1, -1):
        v = vals[i]
        if v:
            out[i] = inv * pref[i] % mod
            inv = inv * v % mod
    return out


# ---------------------------------------------------------------------------
# Byte conversions (ffjavascript toRprLE / toRprBE / toRprLEM)
# ---------------------------------------------------------------------------
def to_le(x: int, n8: int = 32) -> bytes:
    return int(x).to_bytes(n8, "little")


def to_be(x: int, n8: int = 32) -> bytes:
    return int(x).to_bytes(n8, "big")


def from_le(b: bytes) -> int:
    return int.from_bytes(b, "little")


def to_lem(x: int, mod: int) -> bytes:
    return to_le(x * MONT_R % mod)


def from_lem(b: bytes, mod: int) -> int:
    return from_le(b) * pow(MONT_R, -1, mod) % mod


# ---------------------------------------------------------------------------
# NTT over Fr, natural order in/out (ffjavascript Fr.fft / Fr.ifft)
# fft:  A[i] = sum_j a[j] * w^(i*j),        w = FR_W[log2 N]
# ifft: a[j] = (1/N) sum_i A[i] * w^(-i*j)
# ---------------------------------------------------------------------------
def _log2(n: int) -> int:
    k = n.bit_length() - 1
    if 1 << k != n:
        raise ValueError("size must be a power of two")
    return k


def _ntt_core(a, root):
    n = len(a)
    a = list(a)
    j = 0
    for i in range(1, n):
        bit = n >> 1
        while j & bit:
            j ^= bit
            bit >>= 1
        j |= bit
        if i < j:
            a[i], a[j] = a[j], a[i]
    m = 2
    while m <= n:
        wm = pow(root, n // m, R_MOD)
        half = m >> 1
        tw = [1] * half
        for k in range(1, half):
            tw[k] = tw[k - 1] * wm % R_MOD
        for s in range(0, n, m):
            for k in range(half):
                u = a[s + k]
                v = a[s + k + half] * tw[k] % R_MOD
                a[s + k] = (u + v) % R_MOD
                a[s + k + half] = (u - v) % R_MOD
        m <<= 1
    return a


def fft(a):
    k = _log2(len(a))
    return _ntt_core(a, FR_W[k])


def ifft(a):
    n = len(a)
    k = _log2(n)
    out = _ntt_core(a, fr_inv(FR_W[k]))
    ninv = fr_inv(n)
    return [x * ninv % R_MOD for x in out]


def eval_pol(coefs, x):
    """Horner (snarkjs plonk_prove ``evalPol``)."""
    res = 0
    for c in reversed(coefs):
        res = (res * x + c) % R_MOD
    return res


# ---------------------------------------------------------------------------
# G1: y^2 = x^3 + 3 over Fq. Affine points are (x, y) tuples, infinity = None.
# Jacobian (X, Y, Z) with x = X/Z^2, y = Y/Z^3; infinity has Z = 0.
# ---------------------------------------------------------------------------
G1_B = 3
G1_GEN = (1, 2)
J_INF = (1, 1, 0)


def g1_is_on_curve(pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    return (y * y - x * x * x - G1_B) % P_MOD == 0


def jac_double(p):
    X, Y, Z = p
    if Z == 0 or Y == 0:
        return J_INF
    A = X * X % P_MOD
    B = Y * Y % P_MOD
    C = B * B % P_MOD
    D = 2 * ((X + B) * (X + B) - A - C) % P_MOD
    E = 3 * A % P_MOD
    F = E * E % P_MOD
    X3 = (F - 2 * D) % P_MOD
    Y3 = (E * (D - X3) - 8 * C) % P_MOD
    Z3 = 2 * Y * Z % P_MOD
    return (X3, Y3, Z3)


def jac_add(p, q):
    X1, Y1, Z1 = p
    X2, Y2, Z2 = q
    if Z1 == 0:
        return q
    if Z2 == 0:
        return p
    Z1Z1 = Z1 * Z1 % P_MOD
    Z2Z2 = Z2 * Z2 % P_MOD
    U1 = X1 * Z2Z2 % P_MOD
    U2 = X2 * Z1Z1 % P_MOD
    S1 = Y1 * Z2 * Z2Z2 % P_MOD
    S2 = Y2 * Z1 * Z1Z1 % P_MOD
    if U1 == U2:
        if S1 == S2:
            return jac_double(p)
        return J_INF
    H = (U2 - U1) % P_MOD
    I = 4 * H * H % P_MOD
    J = H * I % P_MOD
    r = 2 * (S2 - S1) % P_MOD
    V = U1 * I % P_MOD
    X3 = (r * r - J - 2 * V) % P_MOD
    Y3 = (r * (V - X3) - 2 * S1 * J) % P_MOD
    Z3 = ((Z1 + Z2) ** 2 - Z1Z1 - Z2Z2) * H % P_MOD
    return (X3, Y3, Z3)


def to_jac(pt):
    if pt is None:
        return J_INF
    return (pt[0], pt[1], 1)


def to_affine(p):
    X, Y, Z = p
    if Z == 0:
        return None
    zi = fq_inv(Z)
    zi2 = zi * zi % P_MOD
    return (X * zi2 % P_MOD, Y * zi2 * zi % P_MOD)


def g1_neg(pt):
    if pt is None:
        return None
    return (pt[0], (-pt[1]) % P_MOD)


def g1_add(a, b):
    return to_affine(jac_add(to_jac(a), to_jac(b)))


def g1_mul(pt, k: int):
    k %= R_MOD
    acc = J_INF
    base = to_jac(pt)
    for bit in bin(k)[2:] if k else "":
        acc = jac_double(acc)
        if bit == "1":
            acc = jac_add(acc, base)
    return to_affine(acc)


def msm(points, scalars, c: int | None = None):
    """Pippenger MSM sum s_i * P_i (ffjavascript ``G1.multiExpAffine``).

    The result is a unique group element, so any correct algorithm matches the
    reference bit-for-bit once converted to affine.
    """
    n = min(len(points), len(scalars))
    if n == 0:
        return None
    if c is None:
        c = max(2, min(12, n.bit_length() - 2))
    nwin = (254 + c - 1) // c
    mask = (1 << c) - 1
    result = J_INF
    for w in range(nwin - 1, -1, -1):
        for _ in range(c):
            result = jac_double(result)
        buckets = [J_INF] * (1 << c)
        shift = w * c
        for i in range(n):
            s = scalars[i] % R_MOD
            d = (s >> shift) & mask
            if d and points[i] is not None:
                buckets[d] = jac_add(buckets[d], to_jac(points[i]))
        run = J_INF
        tot = J_INF
        for d in range(mask, 0, -1):
            run = jac_add(run, buckets[d])
            tot = jac_add(tot, run)
        result = jac_add(result, tot)
    return to_affine(result)


def g1_to_lem(pt) -> bytes:
    """64-byte LEM affine (zkey PTau / header points). Infinity = all zeros."""
    if pt is None:
        return bytes(64)
    return to_lem(pt[0], P_MOD) + to_lem(pt[1], P_MOD)


def g1_from_lem(b: bytes):
    x = from_lem(b[:32], P_MOD)
    y = from_lem(b[32:64], P_MOD)
    if x == 0 and y == 0:
        return None
    return (x, y)


def g1_to_uncompressed(pt) -> bytes:
    """ffjavascript ``G1.toRprUncompressed``: x BE || y BE; infinity -> 0x40 flag."""
    if pt is None:
        b = bytearray(64)
        b[0] = 0x40
        return bytes(b)
    return to_be(pt[0]) + to_be(pt[1])


# ---------------------------------------------------------------------------
# Fq2 = Fq[u]/(u^2 + 1) and G2 (twist y^2 = x^3 + 3/(9+u)), enough for the
# zkey header's X_2 = [tau]_2 and for the pairing verifier.
# ---------------------------------------------------------------------------
def fq2_add(a, b):
    return ((a[0] + b[0]) % P_MOD, (a[1] + b[1]) % P_MOD)


def fq2_sub(a, b):
    return ((a[0] - b[0]) % P_MOD, (a[1] - b[1]) % P_MOD)


def fq2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P_MOD, (a[0] * b[1] + a[1] * b[0]) % P_MOD)


def fq2_inv(a):
    d = fq_inv((a[0] * a[0] + a[1] * a[1]) % P_MOD)
    return (a[0] * d % P_MOD, (-a[1]) * d % P_MOD)


FQ2_ZERO = (0, 0)
FQ2_ONE = (1, 0)
G2_B = fq2_mul((3, 0), fq2_inv((9, 1)))
G2_GEN = (
    (10857046999023057135944570762232829481370756359578518086990519993285655852781,
     11559732032986387107991004021392285783925812861821192530917403151452391805634),
    (8495653923123431417604973247489272438418190587263600148770280649306958101930,
     4082367875863433681332203403145435568316851327593401208105741076214120093531),
)


def g2_is_on_curve(pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    lhs = fq2_mul(y, y)
    rhs = fq2_add(fq2_mul(fq2_mul(x, x), x), G2_B)
    return lhs == rhs


def g2_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    (x1, y1), (x2, y2) = a, b
    if x1 == x2:
        if y1 == y2:
            return g2_double(a)
        return None
    lam = fq2_mul(fq2_sub(y2, y1), fq2_inv(fq2_sub(x2, x1)))
    x3 = fq2_sub(fq2_sub(fq2_mul(lam, lam), x1), x2)
    y3 = fq2_sub(fq2_mul(lam, fq2_sub(x1, x3)), y1)
    return (x3, y3)


def g2_double(a):
    if a is None:
        return None
    x, y = a
    if y == FQ2_ZERO:
        return None
    lam = fq2_mul(fq2_mul((3, 0), fq2_mul(x, x)), fq2_inv(fq2_add(y, y)))
    x3 = fq2_sub(fq2_mul(lam, lam), fq2_add(x, x))
    y3 = fq2_sub(fq2_mul(lam, fq2_sub(x, x3)), y)
    return (x3, y3)


def g2_neg(a):
    if a is None:
        return None
    return (a[0], ((-a[1][0]) % P_MOD, (-a[1][1]) % P_MOD))


def g2_mul(pt, k: int):
    k %= R_MOD
    acc = None
    for bit in bin(k)[2:] if k else "":
        acc = g2_double(acc)
        if bit == "1":
            acc = g2_add(acc, pt)
    return acc


def g2_to_lem(pt) -> bytes:
    if pt is None:
        return bytes(128)
    (x0, x1), (y0, y1) = pt
    return to_lem(x0, P_MOD) + to_lem(x1, P_MOD) + to_lem(y0, P_MOD) + to_lem(y1, P_MOD)


def g2_from_lem(b: bytes):
    vals = [from_lem(b[i * 32:(i + 1) * 32], P_MOD) for i in range(4)]
    if not any(vals):
        return None
    return ((vals[0], vals[1]), (vals[2], vals[3]))
