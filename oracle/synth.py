"""Seeded synthetic PLONK circuits (stand-in for the absent nzcp_live.r1cs).

TEST INFRASTRUCTURE ONLY (see ``oracle/bn254.py`` header).

The real ``nzcp_live_final.zkey`` (b2sum at ``/root/reference/README.md:43``)
and its r1cs/ptau cannot be built offline (circom, snarkjs and the ptau are
[EXT], SURVEY.md §7 "Hard parts"). SURVEY.md §8d config 3 therefore
prescribes a *synthetic satisfied circuit* with a seeded tau. This module
defines that circuit family bit-exactly; the HIP library's
``nzcb_synth_setup`` (``nzcb-circom_amd/csrc/synth.hip``) implements the same
generator and ``tests/test_gpu_synth.py`` checks the two agree byte for
byte on the zkey and wtns they emit.

Gate shape follows what snarkjs ``plonk setup`` emits from an r1cs
(SURVEY.md §8a row a3): ``nPublic`` leading public-input gates
``[s, 0, 0 | qm=0, ql=1, qr=0, qo=0, qc=0]``, then arithmetic gates
``qm·a·b + ql·a + qr·b + qo·c + qc = 0`` whose wires reuse earlier signals
(copy constraints), a fraction of them reading an *internal* signal produced
by the additions section (``int = ac·w[ai] + bc·w[bi]``), and padding up to
the domain wired to signal 0 with all-zero selectors.

RNG: xoshiro256** seeded by four splitmix64 outputs. Field draws take four
u64 words little-endian, mask to 254 bits, reject >= r.
"""
from __future__ import annotations

from .bn254 import R_MOD

_M64 = (1 << 64) - 1


class Xoshiro256ss:
    def __init__(self, seed: int):
        x = seed & _M64
        s = []
        for _ in range(4):
            x = (x + 0x9E3779B97F4A7C15) & _M64
            z = x
            z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
            z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
            s.append(z ^ (z >> 31))
        self.s = s

    def next(self) -> int:
        s = self.s
        result = (((s[1] * 5) & _M64) << 7 | ((s[1] * 5) & _M64) >> 57) & _M64
        result = (result * 9) & _M64
        t = (s[1] << 17) & _M64
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = ((s[3] << 45) | (s[3] >> 19)) & _M64
        return result

    def fr(self) -> int:
        while True:
            v = self.next() | (self.next() << 64) | (self.next() << 128) | (self.next() << 192)
            v &= (1 << 254) - 1
            if v < R_MOD:
                return v

    def below(self, m: int) -> int:
        return self.next() % m


def default_n_constraints(power: int) -> int:
    n = 1 << power
    return n - max(1, n >> 5)


def synth_circuit(power: int, n_public: int = 3, n_inputs: int = 8, seed: int = 0x6E7A6362,
                  n_constraints: int | None = None, free_public: bool = False):
    """Return a dict describing a satisfied circuit plus its full witness.

    Keys: ``constraints`` (list of (sa, sb, sc, qm, ql, qr, qo, qc)),
    ``additions`` (ai, bi, ac, bc), ``witness`` (file witness, w[0] = 1),
    ``nVars``, ``nAdditions``, ``nPublic``. With ``free_public`` the public signals
    are left out of the wire pool (NZCB_SYNTH_FREE_PUBLIC), so they sit on their
    public-input gate only and any public values keep the circuit satisfied.
    """
    n = 1 << power
    if n_constraints is None:
        n_constraints = default_n_constraints(power)
    if not (n_public + n_inputs <= n_constraints <= n):
        raise ValueError("bad synthetic circuit size")
    rng = Xoshiro256ss(seed)
    INTERNAL = 1 << 31
    wit = [1]                       # signal 0: the constant-one signal
    vals = {}                       # ref -> value (signal 0 evaluates to 0 in the prover)
    for _ in range(n_public + n_inputs):
        v = rng.fr()
        vals[len(wit)] = v
        wit.append(v)
    internal = []
    additions = []
    pool = list(range(1 + n_public if free_public else 1, 1 + n_public + n_inputs))
    unused = list(range(1 + n_public, 1 + n_public + n_inputs))
    unused_pos = 0

    def pick():
        nonlocal unused_pos
        if unused_pos < len(unused):
            r = unused[unused_pos]
            unused_pos += 1
            return r
        return pool[rng.below(len(pool))]

    cons = []
    for s in range(1, n_public + 1):
        cons.append((s, 0, 0, 0, 1, 0, 0, 0))
    for _ in range(n_constraints - n_public):
        kind = rng.below(8)
        if kind == 7 and unused_pos < len(unused):
            kind = 0    # additions read only signals that already sit on a gate wire
        a = pick()
        b = pick()
        if kind == 7:
            x = pick()
            y = pick()
            ac = rng.fr()
            bc = rng.fr()
            t = INTERNAL | len(internal)
            tv = (ac * vals[x] + bc * vals[y]) % R_MOD
            internal.append(tv)
            vals[t] = tv
            additions.append((x, y, ac, bc))
            a = t
        qm = rng.fr()
        ql = rng.fr()
        qr = rng.fr()
        va, vb = vals[a], vals[b]
        if kind in (5, 6):
            c = pick()
            qo = rng.fr()
            qc = (-(qm * va * vb + ql * va + qr * vb + qo * vals[c])) % R_MOD
        else:
            qo = R_MOD - 1
            qc = rng.fr()
            vc = (qm * va * vb + ql * va + qr * vb + qc) % R_MOD
            c = len(wit)
            wit.append(vc)
            vals[c] = vc
            pool.append(c)
        cons.append((a, b, c, qm, ql, qr, qo, qc))

    n_wit = len(wit)

    def res(ref):
        return n_wit + (ref & ~INTERNAL) if ref & INTERNAL else ref

    cons = [(res(a), res(b), res(c), *q) for (a, b, c, *q) in cons]
    additions = [(res(x), res(y), ac, bc) for (x, y, ac, bc) in additions]
    return {
        "power": power,
        "constraints": cons,
        "additions": additions,
        "witness": wit,
        "nVars": n_wit + len(internal),
        "nAdditions": len(internal),
        "nPublic": n_public,
    }


def fixed_blinding(i: int) -> int:
    """b_i = SHA-256("nzcb-b" || i) mod r, i = 1..11."""
    import hashlib
    return int.from_bytes(hashlib.sha256(b"nzcb-b" + bytes([i])).digest(), "big") % R_MOD


def fixed_blindings():
    return [fixed_blinding(i) for i in range(1, 12)]
