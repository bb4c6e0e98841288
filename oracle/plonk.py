"""PLONK setup / prove / verify — the CPU oracle for the HIP prover.

TEST INFRASTRUCTURE ONLY (see ``oracle/bn254.py`` header).

PARITY UNPINNED against snarkjs: the prover the reference calls
(``snarkjs@0.4.12`` ``plonk_prove.js`` / ``plonk_setup.js`` / ``plonk_verify.js``,
``/root/reference/yarn.lock:7279-7292``, used at ``/root/reference/Makefile:54-62``)
is [EXT] and absent from the container; no reference test pins proof bytes
(SURVEY.md §8c). This file restates the algorithm as specified in
SURVEY.md §8a rows a3-a12 and pins itself through the verifier below
(algebraic identity + KZG openings checked with the known setup trapdoor tau,
and the optimal-ate pairing check in ``oracle/pairing.py``).

Every function names the SURVEY row it restates.
"""
from __future__ import annotations

from . import bn254 as bn
from .bn254 import R_MOD, FR_W, fr_inv, fft, ifft, eval_pol
from .keccak import keccak256

K1 = 2
K2 = 3
N_BLIND = 11


# ---------------------------------------------------------------------------
# Setup (snarkjs 0.4 plonk_setup restated)
# ---------------------------------------------------------------------------
def _p4(evals_n):
    """writeP4: coefficients = ifft(evals on n); evals4 = fft(coefs || 0^{3n})."""
    n = len(evals_n)
    coefs = ifft(evals_n)
    evals4 = fft(coefs + [0] * (3 * n))
    return coefs, evals4


def ptau_points(tau: int, count: int):
    pts = []
    t = 1
    acc_gen = bn.G1_GEN
    for _ in range(count):
        pts.append(bn.g1_mul(acc_gen, t))
        t = t * tau % R_MOD
    return pts


def setup(circuit: dict, tau: int, ptau=None) -> dict:
    power = circuit["power"]
    n = 1 << power
    cons = circuit["constraints"]
    nvars = circuit["nVars"]
    npub = circuit["nPublic"]
    w = FR_W[power]
    if ptau is None:
        ptau = ptau_points(tau, n + 6)
    zk = {
        "nVars": nvars, "nPublic": npub, "domainSize": n, "power": power,
        "nAdditions": circuit["nAdditions"], "nConstraints": len(cons),
        "k1": K1, "k2": K2, "additions": list(circuit["additions"]),
        "aMap": [c[0] for c in cons], "bMap": [c[1] for c in cons], "cMap": [c[2] for c in cons],
        "ptau": ptau,
    }
    for j, name in enumerate(("qm", "ql", "qr", "qo", "qc")):
        col = [0] * n
        for i, c in enumerate(cons):
            col[i] = c[3 + j] % R_MOD
        zk[name] = _p4(col)
    # buildSigma: each position points at the previous appearance of its signal
    sigma = [0] * (3 * n)
    last = {}
    first = {}
    wi = 1
    for i in range(n):
        sig = cons[i][:3] if i < len(cons) else (0, 0, 0)
        for k, s in enumerate(sig):
            p = k * n + i
            if s not in last:
                first[s] = p
            else:
                sigma[p] = last[s]
            last[s] = wi * (1, K1, K2)[k] % R_MOD
        wi = wi * w % R_MOD
    for s in range(nvars):
        if s not in first:
            raise ValueError("Variable not used")
        sigma[first[s]] = last[s]
    zk["sigma"] = [_p4(sigma[k * n:(k + 1) * n]) for k in range(3)]
    zk["lagrange"] = []
    for j in range(max(npub, 1)):
        e = [0] * n
        e[j] = 1
        zk["lagrange"].append(_p4(e))
    base = ptau[:n]
    for name, coefs in (("Qm", zk["qm"][0]), ("Ql", zk["ql"][0]), ("Qr", zk["qr"][0]),
                        ("Qo", zk["qo"][0]), ("Qc", zk["qc"][0]), ("S1", zk["sigma"][0][0]),
                        ("S2", zk["sigma"][1][0]), ("S3", zk["sigma"][2][0])):
        zk[name] = bn.msm(base, coefs)
    zk["X_2"] = bn.g2_mul(bn.G2_GEN, tau)
    return zk


# ---------------------------------------------------------------------------
# Prover (snarkjs 0.4.12 plonk_prove restated)
# ---------------------------------------------------------------------------
class ProverError(Exception):
    pass


def hash_to_fr(data: bytes) -> int:
    """hashToFr: keccak256, big-endian integer, reduced mod r."""
    return int.from_bytes(keccak256(data), "big") % R_MOD


def _fr_be(x: int) -> bytes:
    return bn.to_be(x % R_MOD)


def _div_pol1(P, d):
    """divPol1: quotient of P by (X - d); last coefficient of the result is 0."""
    n = len(P)
    res = [0] * n
    res[n - 2] = P[n - 1]
    for i in range(n - 3, -1, -1):
        res[i] = (P[i + 1] + d * res[i + 1]) % R_MOD
    if P[0] % R_MOD != (-d * res[0]) % R_MOD:
        raise ProverError("Polinomial does not divide")
    return res


def _to4t(A, pz):
    """to4T: coefficients p = ifft(A) blinded with (sum pz_i X^i)(X^n - 1); A4 = fft(p || 0^3n)."""
    n = len(A)
    a = ifft(A)
    A4 = fft(a + [0] * (3 * n))
    a1 = a + [0] * len(pz)
    for i, b in enumerate(pz):
        a1[n + i] = (a1[n + i] + b) % R_MOD
        a1[i] = (a1[i] - b) % R_MOD
    return a1, A4


def prove(zk: dict, witness, blinding=None, transcript_pub: bool = True, trace: dict | None = None):
    """Return (proof, public_signals) with proof as a dict of ints / affine tuples.

    ``blinding``: list of 11 Fr (b1..b11); default all-zero (deterministic).
    ``transcript_pub``: include the public inputs in the beta transcript
    (SURVEY.md §8a row a8 spec); False = A||B||C only.
    """
    n = zk["domainSize"]
    power = zk["power"]
    npub = zk["nPublic"]
    nvars = zk["nVars"]
    nadd = zk["nAdditions"]
    if len(witness) != nvars - nadd:
        raise ProverError(f"Invalid witness length. Circuit: {nvars}, witness: {len(witness)}, {nadd}")
    w = list(witness)
    w[0] = 0                                   # "First element in plonk is not used"
    b = [0] + list(blinding if blinding is not None else [0] * N_BLIND)
    if len(b) != N_BLIND + 1:
        raise ValueError("blinding must have 11 elements")
    nwit = nvars - nadd
    internal = [0] * nadd

    def get_w(idx):
        if idx < nwit:
            return w[idx]
        if idx < nvars:
            return internal[idx - nwit]
        return 0

    # a4: calculateAdditions
    for i, (ai, bi, ac, bc) in enumerate(zk["additions"]):
        internal[i] = (ac * get_w(ai) + bc * get_w(bi)) % R_MOD

    # a5: buildABC
    nc = zk["nConstraints"]
    A = [0] * n
    B = [0] * n
    C = [0] * n
    for i in range(nc):
        A[i] = get_w(zk["aMap"][i])
        B[i] = get_w(zk["bMap"][i])
        C[i] = get_w(zk["cMap"][i])
    ptau = zk["ptau"]

    def exp_tau(coefs):
        return bn.msm(ptau[:len(coefs)], coefs)

    proof = {}
    ch = {}
    # round 1 (a6, a7)
    pol_a, A4 = _to4t(A, [b[2], b[1]])
    pol_b, B4 = _to4t(B, [b[4], b[3]])
    pol_c, C4 = _to4t(C, [b[6], b[5]])
    proof["A"] = exp_tau(pol_a)
    proof["B"] = exp_tau(pol_b)
    proof["C"] = exp_tau(pol_c)

    # round 2 (a8)
    t1 = b""
    if transcript_pub:
        t1 += b"".join(_fr_be(A[i]) for i in range(npub))
    t1 += bn.g1_to_uncompressed(proof["A"]) + bn.g1_to_uncompressed(proof["B"]) + bn.g1_to_uncompressed(proof["C"])
    ch["beta"] = beta = hash_to_fr(t1)
    ch["gamma"] = gamma = hash_to_fr(_fr_be(beta))
    s_evals = [zk["sigma"][k][1] for k in range(3)]
    wn = FR_W[power]
    num = [1] * n
    den = [1] * n
    wi = 1
    for i in range(n):
        bw = beta * wi % R_MOD
        nn = (A[i] + bw + gamma) * (B[i] + K1 * bw + gamma) % R_MOD * (C[i] + K2 * bw + gamma) % R_MOD
        dd = ((A[i] + beta * s_evals[0][4 * i] + gamma) * (B[i] + beta * s_evals[1][4 * i] + gamma) % R_MOD
              * (C[i] + beta * s_evals[2][4 * i] + gamma)) % R_MOD
        num[(i + 1) % n] = num[i] * nn % R_MOD
        den[(i + 1) % n] = den[i] * dd % R_MOD
        wi = wi * wn % R_MOD
    deninv = bn.batch_inverse(den)
    Z = [num[i] * deninv[i] % R_MOD for i in range(n)]
    if Z[0] != 1:
        raise ProverError("Copy constraints does not match")
    pol_z, Z4 = _to4t(Z, [b[9], b[8], b[7]])
    proof["Z"] = exp_tau(pol_z)

    # round 3 (a9)
    ch["alpha"] = alpha = hash_to_fr(bn.g1_to_uncompressed(proof["Z"]))
    alpha2 = alpha * alpha % R_MOD
    w2 = FR_W[2]
    Z1 = [0, (-1 + w2) % R_MOD, (-2) % R_MOD, (-1 - w2) % R_MOD]
    Z2 = [0, (-2 * w2) % R_MOD, 4, (2 * w2) % R_MOD]
    Z3 = [0, (2 + 2 * w2) % R_MOD, (-8) % R_MOD, (2 - 2 * w2) % R_MOD]
    qm4, ql4, qr4, qo4, qc4 = (zk[k][1] for k in ("qm", "ql", "qr", "qo", "qc"))
    lag4 = [zk["lagrange"][j][1] for j in range(len(zk["lagrange"]))]
    n4 = 4 * n
    w4 = FR_W[power + 2]
    T = [0] * n4
    Tz = [0] * n4
    wi = 1
    for i in range(n4):
        a, bb, c, z = A4[i], B4[i], C4[i], Z4[i]
        zw = Z4[(i + 4) % n4]
        s1, s2, s3 = s_evals[0][i], s_evals[1][i], s_evals[2][i]
        ap = (b[2] + b[1] * wi) % R_MOD
        bp = (b[4] + b[3] * wi) % R_MOD
        cp = (b[6] + b[5] * wi) % R_MOD
        wi2 = wi * wi % R_MOD
        zp = (b[7] * wi2 + b[8] * wi + b[9]) % R_MOD
        wW = wi * wn % R_MOD
        wW2 = wW * wW % R_MOD
        zWp = (b[7] * wW2 + b[8] * wW + b[9]) % R_MOD
        pl = 0
        for j in range(npub):
            pl = (pl - lag4[j][i] * A[j]) % R_MOD
        p = i % 4
        # e1 (gate) and its Z_H-quotient part via mul2
        e1 = a * bb % R_MOD
        e1z = (a * bp + ap * bb) % R_MOD
        if p:
            e1z = (e1z + Z1[p] * (ap * bp)) % R_MOD
        e1 = e1 * qm4[i] % R_MOD
        e1z = e1z * qm4[i] % R_MOD
        e1 = (e1 + a * ql4[i] + bb * qr4[i] + c * qo4[i] + pl + qc4[i]) % R_MOD
        e1z = (e1z + ap * ql4[i] + bp * qr4[i] + cp * qo4[i]) % R_MOD
        betaw = beta * wi % R_MOD
        e2, e2z = _mul4((a + betaw + gamma) % R_MOD, (bb + betaw * K1 + gamma) % R_MOD,
                        (c + betaw * K2 + gamma) % R_MOD, z, ap, bp, cp, zp, p, Z1, Z2, Z3)
        e2 = e2 * alpha % R_MOD
        e2z = e2z * alpha % R_MOD
        e3, e3z = _mul4((a + beta * s1 + gamma) % R_MOD, (bb + beta * s2 + gamma) % R_MOD,
                        (c + beta * s3 + gamma) % R_MOD, zw, ap, bp, cp, zWp, p, Z1, Z2, Z3)
        e3 = e3 * alpha % R_MOD
        e3z = e3z * alpha % R_MOD
        l1 = lag4[0][i]
        e4 = (z - 1) * l1 % R_MOD * alpha2 % R_MOD
        e4z = zp * l1 % R_MOD * alpha2 % R_MOD
        T[i] = (e1 + e2 - e3 + e4) % R_MOD
        Tz[i] = (e1z + e2z - e3z + e4z) % R_MOD
        wi = wi * w4 % R_MOD
    t = ifft(T)
    for i in range(n):
        t[i] = (-t[i]) % R_MOD
    for i in range(n, n4):
        t[i] = (t[i - n] - t[i]) % R_MOD
        if i > 3 * n - 4 and t[i] != 0:
            raise ProverError("T Polynomial is not divisible")
    tz = ifft(Tz)
    for i in range(n4):
        if i > 3 * n + 5:
            if tz[i] != 0:
                raise ProverError("Tz Polynomial is not well calculated")
        else:
            t[i] = (t[i] + tz[i]) % R_MOD
    pol_t = t[:3 * n + 6]
    proof["T1"] = exp_tau(t[:n])
    proof["T2"] = exp_tau(t[n:2 * n])
    proof["T3"] = exp_tau(t[2 * n:3 * n + 6])

    # round 4 (a10)
    ch["xi"] = xi = hash_to_fr(bn.g1_to_uncompressed(proof["T1"]) + bn.g1_to_uncompressed(proof["T2"])
                               + bn.g1_to_uncompressed(proof["T3"]))
    pol_s1 = zk["sigma"][0][0]
    pol_s2 = zk["sigma"][1][0]
    pol_s3 = zk["sigma"][2][0]
    ev = {}
    ev["a"] = eval_pol(pol_a, xi)
    ev["b"] = eval_pol(pol_b, xi)
    ev["c"] = eval_pol(pol_c, xi)
    ev["s1"] = eval_pol(pol_s1, xi)
    ev["s2"] = eval_pol(pol_s2, xi)
    ev["t"] = eval_pol(pol_t, xi)
    ev["zw"] = eval_pol(pol_z, xi * wn % R_MOD)
    coef_ab = ev["a"] * ev["b"] % R_MOD
    betaxi = beta * xi % R_MOD
    e2 = ((ev["a"] + betaxi + gamma) * (ev["b"] + betaxi * K1 + gamma) % R_MOD
          * (ev["c"] + betaxi * K2 + gamma) % R_MOD * alpha) % R_MOD
    e3 = ((ev["a"] + beta * ev["s1"] + gamma) * (ev["b"] + beta * ev["s2"] + gamma) % R_MOD
          * beta % R_MOD * ev["zw"] % R_MOD * alpha) % R_MOD
    xim = pow(xi, n, R_MOD)
    ch["xim"] = xim
    eval_l1 = (xim - 1) * fr_inv((xi - 1) * n % R_MOD) % R_MOD
    e4 = eval_l1 * alpha2 % R_MOD
    coefz = (e2 + e4) % R_MOD
    qm, ql, qr, qo, qc = (zk[k][0] for k in ("qm", "ql", "qr", "qo", "qc"))
    pol_r = [0] * (n + 3)
    for i in range(n + 3):
        v = coefz * pol_z[i]
        if i < n:
            v += coef_ab * qm[i] + ev["a"] * ql[i] + ev["b"] * qr[i] + ev["c"] * qo[i] + qc[i] - e3 * pol_s3[i]
        pol_r[i] = v % R_MOD
    ev["r"] = eval_pol(pol_r, xi)

    # round 5 (a11)
    t5 = b"".join(_fr_be(ev[k]) for k in ("a", "b", "c", "s1", "s2", "zw", "r"))
    v = [0] * 7
    v[1] = hash_to_fr(t5)
    for i in range(2, 7):
        v[i] = v[i - 1] * v[1] % R_MOD
    ch["v"] = v
    xi2m = xim * xim % R_MOD
    pol_wxi = [0] * (n + 6)
    for i in range(n + 6):
        acc = xi2m * t[2 * n + i]
        if i < n:
            acc += xim * t[n + i] + t[i]
        if i < n + 3:
            acc += v[1] * pol_r[i]
        if i < n + 2:
            acc += v[2] * pol_a[i] + v[3] * pol_b[i] + v[4] * pol_c[i]
        if i < n:
            acc += v[5] * pol_s1[i] + v[6] * pol_s2[i]
        pol_wxi[i] = acc % R_MOD
    pol_wxi[0] = (pol_wxi[0] - ev["t"] - v[1] * ev["r"] - v[2] * ev["a"] - v[3] * ev["b"] - v[4] * ev["c"]
                  - v[5] * ev["s1"] - v[6] * ev["s2"]) % R_MOD
    pol_wxi = _div_pol1(pol_wxi, xi)
    proof["Wxi"] = exp_tau(pol_wxi)
    pol_wxiw = list(pol_z[:n + 3])
    pol_wxiw[0] = (pol_wxiw[0] - ev["zw"]) % R_MOD
    pol_wxiw = _div_pol1(pol_wxiw, xi * wn % R_MOD)
    proof["Wxiw"] = exp_tau(pol_wxiw)

    for k in ("a", "b", "c", "s1", "s2", "zw", "r"):
        proof["eval_" + k] = ev[k]
    public = [witness[i] % R_MOD for i in range(1, npub + 1)]
    if trace is not None:
        trace.update(ch)
        trace["eval_t"] = ev["t"]
        trace.update({"pol_a": pol_a, "pol_b": pol_b, "pol_c": pol_c, "pol_z": pol_z, "pol_t": pol_t,
                      "pol_r": pol_r, "pol_wxi": pol_wxi, "pol_wxiw": pol_wxiw, "A4": A4, "Z4": Z4,
                      "T": T, "Tz": Tz, "Z": Z, "A": A, "B": B, "C": C})
    return proof, public


def _mul4(a, b, c, d, ap, bp, cp, dp, p, Z1, Z2, Z3):
    """mul4: product of 4 blinded factors split into (value, Z_H-quotient part)."""
    a_b = a * b % R_MOD
    a_bp = a * bp % R_MOD
    ap_b = ap * b % R_MOD
    ap_bp = ap * bp % R_MOD
    c_d = c * d % R_MOD
    c_dp = c * dp % R_MOD
    cp_d = cp * d % R_MOD
    cp_dp = cp * dp % R_MOD
    r = a_b * c_d % R_MOD
    a0 = (ap_b * c_d + a_bp * c_d + a_b * cp_d + a_b * c_dp) % R_MOD
    a1 = (ap_bp * c_d + ap_b * cp_d + ap_b * c_dp + a_bp * cp_d + a_bp * c_dp + a_b * cp_dp) % R_MOD
    a2 = (a_bp * cp_dp + ap_b * cp_dp + ap_bp * c_dp + ap_bp * cp_d) % R_MOD
    a3 = ap_bp * cp_dp % R_MOD
    rz = a0
    if p:
        rz = (rz + Z1[p] * a1 + Z2[p] * a2 + Z3[p] * a3) % R_MOD
    return r, rz


# ---------------------------------------------------------------------------
# Serialisation of proofs (binary C-ABI layout and snarkjs JSON)
# ---------------------------------------------------------------------------
PROOF_POINTS = ("A", "B", "C", "Z", "T1", "T2", "T3", "Wxi", "Wxiw")
PROOF_EVALS = ("eval_a", "eval_b", "eval_c", "eval_s1", "eval_s2", "eval_zw", "eval_r")
PROOF_BYTES = 9 * 64 + 7 * 32


def proof_to_bytes(proof) -> bytes:
    out = b""
    for k in PROOF_POINTS:
        p = proof[k]
        out += bytes(64) if p is None else bn.to_le(p[0]) + bn.to_le(p[1])
    for k in PROOF_EVALS:
        out += bn.to_le(proof[k])
    return out


def proof_from_bytes(data: bytes):
    proof = {}
    for i, k in enumerate(PROOF_POINTS):
        x = bn.from_le(data[64 * i:64 * i + 32])
        y = bn.from_le(data[64 * i + 32:64 * i + 64])
        proof[k] = None if (x == 0 and y == 0) else (x, y)
    for j, k in enumerate(PROOF_EVALS):
        o = 9 * 64 + 32 * j
        proof[k] = bn.from_le(data[o:o + 32])
    return proof


def proof_to_json_obj(proof):
    """snarkjs key order: A B C Z T1 T2 T3 evals Wxi Wxiw protocol curve (eval_t deleted)."""
    def g1(p):
        return ["0", "1", "0"] if p is None else [str(p[0]), str(p[1]), "1"]
    out = {}
    for k in ("A", "B", "C", "Z", "T1", "T2", "T3"):
        out[k] = g1(proof[k])
    for k in PROOF_EVALS:
        out[k] = str(proof[k])
    out["Wxi"] = g1(proof["Wxi"])
    out["Wxiw"] = g1(proof["Wxiw"])
    out["protocol"] = "plonk"
    out["curve"] = "bn128"
    return out


# ---------------------------------------------------------------------------
# Verifier (snarkjs 0.4.x plonk_verify restated)
# ---------------------------------------------------------------------------
def verifier_challenges(proof, public, transcript_pub=True):
    ch = {}
    t1 = b"".join(_fr_be(x) for x in public) if transcript_pub else b""
    t1 += b"".join(bn.g1_to_uncompressed(proof[k]) for k in ("A", "B", "C"))
    ch["beta"] = hash_to_fr(t1)
    ch["gamma"] = hash_to_fr(_fr_be(ch["beta"]))
    ch["alpha"] = hash_to_fr(bn.g1_to_uncompressed(proof["Z"]))
    ch["xi"] = hash_to_fr(b"".join(bn.g1_to_uncompressed(proof[k]) for k in ("T1", "T2", "T3")))
    v = [0] * 7
    v[1] = hash_to_fr(b"".join(_fr_be(proof[k]) for k in PROOF_EVALS))
    for i in range(2, 7):
        v[i] = v[i - 1] * v[1] % R_MOD
    ch["v"] = v
    ch["u"] = hash_to_fr(bn.g1_to_uncompressed(proof["Wxi"]) + bn.g1_to_uncompressed(proof["Wxiw"]))
    return ch


def verify_prepare(vk: dict, public, proof, transcript_pub=True):
    """Compute the two G1 points of the final KZG pairing check.

    Returns (ch, lhs, rhs) such that a valid proof satisfies
    e(lhs, [tau]_2) == e(rhs, [1]_2), i.e. tau*lhs == rhs when tau is known.
    """
    n = vk["domainSize"]
    power = n.bit_length() - 1
    wn = FR_W[power]
    ch = verifier_challenges(proof, public, transcript_pub)
    beta, gamma, alpha, xi, v, u = ch["beta"], ch["gamma"], ch["alpha"], ch["xi"], ch["v"], ch["u"]
    alpha2 = alpha * alpha % R_MOD
    xin = pow(xi, n, R_MOD)
    zh = (xin - 1) % R_MOD
    L = []
    wpow = 1
    for i in range(max(len(public), 1)):
        L.append(wpow * zh % R_MOD * fr_inv(n * (xi - wpow) % R_MOD) % R_MOD)
        wpow = wpow * wn % R_MOD
    pl = sum(-L[i] * public[i] for i in range(len(public))) % R_MOD   # PI(xi)
    ea, eb, ec = proof["eval_a"], proof["eval_b"], proof["eval_c"]
    es1, es2, ezw, er = proof["eval_s1"], proof["eval_s2"], proof["eval_zw"], proof["eval_r"]
    num = (er + pl - (ea + beta * es1 + gamma) * (eb + beta * es2 + gamma) % R_MOD * (ec + gamma) % R_MOD
           * ezw % R_MOD * alpha - L[0] * alpha2) % R_MOD
    t = num * fr_inv(zh) % R_MOD
    ch["eval_t"] = t
    betaxi = beta * xi % R_MOD
    e2 = ((ea + betaxi + gamma) * (eb + betaxi * K1 + gamma) % R_MOD * (ec + betaxi * K2 + gamma) % R_MOD
          * alpha) % R_MOD
    e4 = L[0] * alpha2 % R_MOD
    e3 = ((ea + beta * es1 + gamma) * (eb + beta * es2 + gamma) % R_MOD * beta % R_MOD * ezw % R_MOD
          * alpha) % R_MOD
    v1 = v[1]
    terms = [
        (vk["Qm"], ea * eb % R_MOD * v1), (vk["Ql"], ea * v1), (vk["Qr"], eb * v1), (vk["Qo"], ec * v1),
        (vk["Qc"], v1), (proof["Z"], ((e2 + e4) * v1 + u) % R_MOD), (vk["S3"], (-e3 * v1) % R_MOD),
    ]
    D = bn.msm([p for p, _ in terms], [s for _, s in terms], c=2)
    terms_f = [
        (proof["T1"], 1), (proof["T2"], xin), (proof["T3"], xin * xin % R_MOD), (D, 1),
        (proof["A"], v[2]), (proof["B"], v[3]), (proof["C"], v[4]), (vk["S1"], v[5]), (vk["S2"], v[6]),
    ]
    F = bn.msm([p for p, _ in terms_f], [s for _, s in terms_f], c=2)
    e = (t + v[1] * er + v[2] * ea + v[3] * eb + v[4] * ec + v[5] * es1 + v[6] * es2 + u * ezw) % R_MOD
    E = bn.g1_mul(bn.G1_GEN, e)
    lhs = bn.g1_add(proof["Wxi"], bn.g1_mul(proof["Wxiw"], u))
    rhs = bn.msm([proof["Wxi"], proof["Wxiw"], F, bn.g1_neg(E)],
                 [xi, u * xi % R_MOD * wn % R_MOD, 1, 1], c=2)
    return ch, lhs, rhs


def verify_with_trapdoor(vk: dict, public, proof, tau: int, transcript_pub=True) -> bool:
    """KZG check with the known synthetic-setup trapdoor: tau*lhs == rhs."""
    if any(not bn.g1_is_on_curve(proof[k]) for k in PROOF_POINTS):
        return False
    _, lhs, rhs = verify_prepare(vk, public, proof, transcript_pub)
    return bn.g1_mul(lhs, tau) == rhs


# ---------------------------------------------------------------------------
# verification key, pairing verifier, calldata
# ---------------------------------------------------------------------------
VK_POINTS = ("Qm", "Ql", "Qr", "Qo", "Qc", "S1", "S2", "S3")


def vk_from_zkey(zk: dict) -> dict:
    """snarkjs 0.4.x `zkey export verificationkey` for PLONK (zkey_export_verificationkey.js
    [EXT], run at /root/reference/Makefile:56,61): the header facts and the selector /
    permutation commitments, X_2 = [tau]_2 and the domain generator w."""
    vk = {"protocol": "plonk", "curve": "bn128", "nPublic": zk["nPublic"], "power": zk["power"],
          "k1": zk["k1"], "k2": zk["k2"]}
    for k in VK_POINTS:
        vk[k] = zk[k]
    vk["X_2"] = zk["X_2"]
    vk["w"] = FR_W[zk["power"]]
    vk["domainSize"] = zk["domainSize"]
    return vk


def vk_to_json_obj(vk: dict) -> dict:
    """verification_key.json layout (decimal strings, projective "1" coordinates)."""
    def g1(p):
        return ["0", "1", "0"] if p is None else [str(p[0]), str(p[1]), "1"]

    out = {"protocol": "plonk", "curve": "bn128", "nPublic": vk["nPublic"], "power": vk["power"],
           "k1": str(vk["k1"]), "k2": str(vk["k2"])}
    for k in VK_POINTS:
        out[k] = g1(vk[k])
    (x0, x1), (y0, y1) = vk["X_2"]
    out["X_2"] = [[str(x0), str(x1)], [str(y0), str(y1)], ["1", "0"]]
    out["w"] = str(vk["w"])
    return out


def verify(vk: dict, public, proof, transcript_pub=True) -> bool:
    """snarkjs plonk_verify restated with the pairing: e(-lhs, X_2) * e(rhs, [1]_2) == 1
    (lhs = Wxi + u Wxiw, rhs = xi Wxi + u xi w Wxiw + F - E; see verify_prepare)."""
    from . import pairing
    if any(not bn.g1_is_on_curve(proof[k]) for k in PROOF_POINTS):
        return False
    if any(not 0 <= proof[k] < R_MOD for k in PROOF_EVALS) or any(not 0 <= x < R_MOD for x in public):
        return False
    vk = dict(vk)
    vk.setdefault("domainSize", 1 << vk["power"])
    _, lhs, rhs = verify_prepare(vk, public, proof, transcript_pub)
    return pairing.pairing_check([(bn.g1_neg(lhs), vk["X_2"]), (rhs, bn.G2_GEN)])


def solidity_calldata(proof, public) -> str:
    """snarkjs 0.4.x `zkey export soliditycalldata` for PLONK (plonk_exportsoliditycalldata.js
    [EXT], consumer at /root/reference/Makefile:57,62): "0x" + the 9 points as uncompressed
    big-endian x||y and the 7 evaluations big-endian, then the public signals as 0x-hex."""
    buf = b"".join(bn.g1_to_uncompressed(proof[k]) for k in PROOF_POINTS)
    buf += b"".join(_fr_be(proof[k]) for k in PROOF_EVALS)
    pubs = ",".join('"0x%064x"' % x for x in public)
    return "0x" + buf.hex() + ",[" + pubs + "]"
