"""The three-coset quotient's algebra (csrc/prover.hip Prover::round3_quot3, k_t_combine),
checked with exact integers at n = 16: (i) the six top coefficients of the numerator N,
N[4n + k] = alpha (A B C Z - (A + beta S1)(B + beta S2)(C + beta S3) Z(wX))[4n + k], equal the
host's convolution of the factors' top coefficients (offsets from the top degree, sigma's
four top coefficients, Z(wX)'s w^(2 - u) factors); (ii) t (degree 3n + 5) is rebuilt exactly
from its evaluations on the three cosets c_j H (per-coset inverse transform, untwist c_j^-k,
1/4) and its top six coefficients. The GPU path itself is checked bit for bit by the proof
parity tests (tests/test_gpu_*.py)."""
import random
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.bn254 import R_MOD as r, FR_W, fr_inv  # noqa: E402


def test_three_coset_quotient_algebra():
    random.seed(1)
    power = 4; n = 1 << power; n4 = 4 * n
    w = FR_W[power]; w4 = FR_W[power + 2]; g = 5
    def rnd(k): return [random.randrange(r) for _ in range(k)]
    def pmul(a, b):
        out = [0] * (len(a) + len(b) - 1)
        for i, x in enumerate(a):
            for j, y in enumerate(b): out[i + j] = (out[i + j] + x * y) % r
        return out
    def padd(a, b, sgn=1):
        m = max(len(a), len(b)); a = a + [0] * (m - len(a)); b = b + [0] * (m - len(b))
        return [(x + sgn * y) % r for x, y in zip(a, b)]
    def ev(p, x): 
        acc = 0
        for c in reversed(p): acc = (acc * x + c) % r
        return acc
    A, B, C = rnd(n + 2), rnd(n + 2), rnd(n + 2); Z = rnd(n + 3)
    S = [rnd(n) for _ in range(3)]
    beta, gamma, alpha = rnd(3)
    K1, K2 = 2, 3
    f1 = padd(A, [gamma, beta]); f2 = padd(B, [gamma, beta * K1]); f3 = padd(C, [gamma, beta * K2])
    P1 = pmul(pmul(pmul(f1, f2), f3), Z)
    g1 = padd(padd(A, [x * beta % r for x in S[0]]), [gamma]); g2 = padd(padd(B, [x * beta % r for x in S[1]]), [gamma])
    g3 = padd(padd(C, [x * beta % r for x in S[2]]), [gamma])
    Zw = [Z[j] * pow(w, j, r) % r for j in range(len(Z))]
    P2 = pmul(pmul(pmul(g1, g2), g3), Zw)
    Nperm = [alpha * x % r for x in padd(P1, P2, -1)]
    assert len(Nperm) == 4 * n + 6
    # (i) top coefficients by the host formula
    top = [A[n - 4:n + 2], B[n - 4:n + 2], C[n - 4:n + 2], Z[n - 3:n + 3]]
    sig_top = [S[k][n - 4:n] for k in range(3)]
    wi = fr_inv(w)
    wpow = [w * w % r, w, 1, wi, wi * wi % r, wi * wi * wi % r]
    p1 = [[0] * 6 for _ in range(4)]; p2 = [[0] * 6 for _ in range(4)]
    for u in range(6):
        for f in range(3):
            p1[f][u] = top[f][5 - u]; p2[f][u] = top[f][5 - u]
            if u >= 2: p2[f][u] = (p2[f][u] + beta * sig_top[f][5 - u]) % r
        p1[3][u] = top[3][5 - u]; p2[3][u] = top[3][5 - u] * wpow[u] % r
    def conv(x, y): return [sum(x[u] * y[s - u] for u in range(s + 1)) % r for s in range(6)]
    e3 = conv(conv(conv(p1[0], p1[1]), p1[2]), p1[3]); h3 = conv(conv(conv(p2[0], p2[1]), p2[2]), p2[3])
    q3 = [alpha * (e3[5 - k] - h3[5 - k]) % r for k in range(6)]
    assert q3 == Nperm[4 * n:4 * n + 6], "top coefficients"
    # (ii) reconstruction of a random t of degree 3n + 5 from three cosets + its top 6
    t = rnd(3 * n + 6)
    c = [g * pow(w4, j, r) % r for j in range(3)]
    d = [pow(cj, n, r) for cj in c]
    V = []
    for j in range(3):
        evals = [ev(t, c[j] * pow(w, m, r) % r) for m in range(n)]
        # iNTT_n then untwist c_j^-k and / 4 (itw3 = c_j^-k / 4n, iNTT without 1/n)
        inv4n = fr_inv(4 * n)
        cji = fr_inv(c[j])
        v = [sum(evals[m] * pow(wi, m * k, r) for m in range(n)) % r * pow(cji, k, r) % r * inv4n % r for k in range(n)]
        V.append(v)
    D = d[0]; D3 = pow(D, 3, r); i4 = d[1] * fr_inv(D) % r; quarter = fr_inv(4)
    assert i4 == pow(w4, n, r)
    qq = t[3 * n:3 * n + 6]
    out = [0] * n4
    for k in range(n):
        v0, v1, v2 = V[0][k], V[1][k], V[2][k]
        if k < 6:
            cc = D3 * qq[k] % r * quarter % r
            v0 = (v0 - cc) % r; v1 = (v1 + i4 * cc) % r; v2 = (v2 + cc) % r
        sm = (v0 + v2) % r; dl = (v0 - v2) % r; im = dl * i4 % r; v12 = 2 * v1 % r
        out[k] = (sm + v12 - im) % r
        out[n + k] = dl * 2 % r * fr_inv(D) % r
        out[2 * n + k] = (sm - v12 + im) % r * fr_inv(D * D % r) % r
        out[3 * n + k] = qq[k] if k < 6 else 0
    assert out[:3 * n + 6] == t and all(x == 0 for x in out[3 * n + 6:]), "reconstruction"

