"""BN254 optimal-ate pairing -- TEST INFRASTRUCTURE ONLY (CPU oracle for the PLONK
verifier).

Restates the pairing check that snarkjs 0.4.12 plonk_verify.js [EXT] runs through
ffjavascript 0.2.48 / wasmcurves 0.1.0 (/root/reference/yarn.lock:3905-3913,
8173-8179): e(-(Wxi + u Wxiw), X_2) * e(xi Wxi + u xi w Wxiw + F - E, G2) == 1.
Not on disk, so the published optimal-ate algorithm for BN254 is restated:
  Fq12 = Fq[w] / (w^12 - 18 w^6 + 82), with Fq2 = Fq[u]/(u^2 + 1) embedded by u = w^6 - 9
  (so w^6 = xi = 9 + u), D-type twist E': y^2 = x^3 + 3/xi mapped by (x, y) -> (x w^2, y w^3),
  Miller loop over 6x + 2 (x = 4965661367192848881) with affine Fq2 point arithmetic and
  sparse line evaluation, the two Frobenius corrections Q1 = pi(Q), -Q2 = -pi^2(Q), and
  the final exponentiation to the power (p^12 - 1) / r.
Pinned by bilinearity / non-degeneracy tests and the trapdoor check (tests/test_pairing.py).
"""
from .bn254 import P_MOD as P, R_MOD, fq2_add, fq2_sub, fq2_mul, fq2_inv, G2_GEN, G1_GEN

ATE_LOOP = 29793968203157093288  # 6x + 2
XI = (9, 1)


def fq2_pow(a, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = fq2_mul(r, a)
        a = fq2_mul(a, a)
        e >>= 1
    return r


def fq2_conj(a):
    return (a[0], (-a[1]) % P)


# Frobenius on the twist: pi(x, y) = (conj(x) g12, conj(y) g13); pi^2(x, y) = (x g22, y g23)
G12 = fq2_pow(XI, (P - 1) // 3)
G13 = fq2_pow(XI, (P - 1) // 2)
G22 = fq2_pow(XI, (P * P - 1) // 3)
G23 = fq2_pow(XI, (P * P - 1) // 2)


def f12_one():
    return [1] + [0] * 11


def f12_mul(a, b):
    r = [0] * 23
    for i, x in enumerate(a):
        if x:
            for j, y in enumerate(b):
                r[i + j] += x * y
    for k in range(22, 11, -1):  # w^12 = 18 w^6 - 82
        c = r[k]
        if c:
            r[k - 6] += 18 * c
            r[k - 12] -= 82 * c
    return [v % P for v in r[:12]]


def f12_pow(a, e):
    r = f12_one()
    while e:
        if e & 1:
            r = f12_mul(r, a)
        a = f12_mul(a, a)
        e >>= 1
    return r


def f12_from_fq2(e, k):
    """Fq2 element e = e0 + e1 u times w^k (k + 6 < 12)."""
    r = [0] * 12
    r[k] = (e[0] - 9 * e[1]) % P
    r[k + 6] = e[1] % P
    return r


def _line(T, S, P1):
    """Line through T and S (affine twist points, S == T: tangent) at P1 in G1, as Fq12."""
    xp, yp = P1
    if T[0] == S[0] and fq2_add(T[1], S[1]) == (0, 0):  # vertical: x - xT
        r = [0] * 12
        r[0] = xp % P
        tx = f12_from_fq2(T[0], 2)
        return [(r[i] - tx[i]) % P for i in range(12)]
    if T == S:
        lam = fq2_mul(fq2_mul((3, 0), fq2_mul(T[0], T[0])), fq2_inv(fq2_add(T[1], T[1])))
    else:
        lam = fq2_mul(fq2_sub(S[1], T[1]), fq2_inv(fq2_sub(S[0], T[0])))
    # l(P) = yP - lam xP w + (lam xT - yT) w^3
    r = [0] * 12
    r[0] = yp % P
    a = f12_from_fq2(fq2_mul(lam, ((-xp) % P, 0)), 1)
    b = f12_from_fq2(fq2_sub(fq2_mul(lam, T[0]), T[1]), 3)
    return [(r[i] + a[i] + b[i]) % P for i in range(12)]


def _add(T, S):
    if T is None:
        return S
    if S is None:
        return T
    if T[0] == S[0]:
        if fq2_add(T[1], S[1]) == (0, 0):
            return None
        lam = fq2_mul(fq2_mul((3, 0), fq2_mul(T[0], T[0])), fq2_inv(fq2_add(T[1], T[1])))
    else:
        lam = fq2_mul(fq2_sub(S[1], T[1]), fq2_inv(fq2_sub(S[0], T[0])))
    x3 = fq2_sub(fq2_sub(fq2_mul(lam, lam), T[0]), S[0])
    y3 = fq2_sub(fq2_mul(lam, fq2_sub(T[0], x3)), T[1])
    return (x3, y3)


def miller_loop(Q, P1):
    """f_{6x+2,Q}(P) * l_{R,Q1}(P) * l_{R+Q1,-Q2}(P), without the final exponentiation."""
    if Q is None or P1 is None:
        return f12_one()
    R = Q
    f = f12_one()
    for i in range(63, -1, -1):
        f = f12_mul(f12_mul(f, f), _line(R, R, P1))
        R = _add(R, R)
        if ATE_LOOP >> i & 1:
            f = f12_mul(f, _line(R, Q, P1))
            R = _add(R, Q)
    Q1 = (fq2_mul(fq2_conj(Q[0]), G12), fq2_mul(fq2_conj(Q[1]), G13))
    nQ2 = (fq2_mul(Q[0], G22), fq2_mul(((-Q[1][0]) % P, (-Q[1][1]) % P), G23))
    f = f12_mul(f, _line(R, Q1, P1))
    R = _add(R, Q1)
    f = f12_mul(f, _line(R, nQ2, P1))
    return f


FINAL_EXP = (P ** 12 - 1) // R_MOD


def final_exp(f):
    return f12_pow(f, FINAL_EXP)


def pairing(Q, P1):
    """e(P1, Q) for P1 in G1 (affine ints), Q in G2 (affine Fq2 pairs)."""
    return final_exp(miller_loop(Q, P1))


def pairing_check(pairs):
    """prod e(P_i, Q_i) == 1 for pairs [(P_i in G1, Q_i in G2)]."""
    f = f12_one()
    for p1, q in pairs:
        f = f12_mul(f, miller_loop(q, p1))
    return final_exp(f) == f12_one()


__all__ = ["pairing", "pairing_check", "miller_loop", "final_exp", "G1_GEN", "G2_GEN"]
