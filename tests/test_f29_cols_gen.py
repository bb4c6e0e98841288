"""csrc/f29_cols.h is generated (tools/gen_f29_cols.py): the committed header must be the
generator's current output, and every product column must hold the terms of f29.h's
reference loops (checked here by re-deriving the term multiset per column)."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nzcb-circom_amd")


def _gen():
    return subprocess.run([sys.executable, os.path.join(PKG, "tools", "gen_f29_cols.py")], check=True,
                          capture_output=True, text=True).stdout


def test_header_is_generator_output():
    with open(os.path.join(PKG, "csrc", "f29_cols.h")) as f:
        assert f.read() == _gen()


def _functions(src):
    out = {}
    for m in re.finditer(r"__device__ __forceinline__ \w+ (\w+)\(", src):
        start = m.end()
        end = src.find("\n}\n", start)
        out[m.group(1)] = src[start:end]
    return out


def _asm_terms(body):
    """(accumulator, x expr, y expr) of every mad, statement by statement."""
    stmts = []
    for m in re.finditer(r'asm\("(.*?)"\n\s*: (.*?)\n\s*: (.*?)\n\s*: "vcc"\);', body, re.S):
        lines, outs, ins = m.group(1).split("\\n\\t"), m.group(2), m.group(3)
        naccs = outs.count('"=&v"') + outs.count('"+v"')
        ops = re.findall(r'"[vs]"\(([^()]*(?:\([^()]*\))?[^()]*)\)', ins)
        mads = []
        for ln in lines:
            mm = re.match(r"v_mad_u64_u32 %(\d+), vcc, %(\d+), %(\d+), (?:%\d+|0)", ln)
            if mm:
                mads.append((int(mm.group(1)), ops[int(mm.group(2)) - naccs], ops[int(mm.group(3)) - naccs]))
        stmts.append(mads)
    return stmts


def test_mul29x2_columns_hold_every_product_term():
    f = _functions(_gen())["mul29x2_cols"]
    stmts = _asm_terms(f)
    prod = {}
    for s in stmts:
        for acc, x, y in s:
            if x.startswith("a.v") or x.startswith("c.v"):
                i = int(re.search(r"\[(\d)\]", x).group(1)) + int(re.search(r"\[(\d)\]", y).group(1))
                prod.setdefault((acc, i), set()).add((x, y))
    for i in range(17):
        want_a = {(f"a.v[{j}]", f"b.v[{i - j}]") for j in range(max(0, i - 8), min(i, 8) + 1)}
        want_c = {(f"c.v[{j}]", f"d.v[{i - j}]") for j in range(max(0, i - 8), min(i, 8) + 1)}
        assert prod[(0, i)] == want_a and prod[(1, i)] == want_c
    # Montgomery terms: m_j P_k for every j, k in 0..8, once per chain
    red = [(acc, x, y) for s in stmts for acc, x, y in s if x.startswith(("m[", "n["))]
    assert len(red) == 2 * 81 and len(set(red)) == 2 * 81


# ---- every generated function, executed: a host emulator of the header ------
# The two instructions the header uses, with the column bound checked (an accumulator that
# passed 2^64 would be a wrong product on the GPU): v_mad_u64_u32 d, vcc, x, y, z: d = x y + z;
# v_lshrrev_b64 d, 29, s: d = s >> 29. The C statements between the asm statements (Montgomery
# digits, result limbs, Shoup quotient limbs) are matched by pattern; any other statement fails
# the test, so the emulator cannot silently skip part of a function.
def _consts():
    with open(os.path.join(PKG, "csrc", "f29.h")) as f:
        src = f.read()
    out = {}
    for q in ("Fq29", "Fr29"):
        body = src[src.index(f"struct {q} {{"):]
        body = body[:body.index("\n};")]
        c = {}
        for name, val in re.findall(r"static constexpr uint32_t (\w+) = (0x[0-9a-f]+)u;", body):
            c[name] = int(val, 16)
        assert "MASK = (1u << 29) - 1;" in body
        c["MASK"] = (1 << 29) - 1
        for name, vals in re.findall(r"static constexpr uint32_t (\w+)\[9\] = \{([^}]*)\}", body):
            c[name] = [int(v.strip().rstrip("u"), 16) for v in vals.split(",")]
        out[q] = c
    return out


_P = 21888242871839275222246405745257275088696311157297823662689037894645226208583
_R = 21888242871839275222246405745257275088548364400416034343698204186575808495617


def _val(limbs):
    return sum(v << (29 * i) for i, v in enumerate(limbs))


def _split(x):
    return [(x >> (29 * i)) & ((1 << 29) - 1) for i in range(8)] + [x >> (29 * 8)]


class _Emu:
    def __init__(self, consts, q):
        self.c, self.q = consts, q
        self.env = {}
        self.max_acc = 0

    def get(self, e):
        e = e.strip()
        m = re.fullmatch(r"(\w+)::(\w+)\[(\d)\]", e)
        if m:
            q = self.q if m.group(1) == "Q" else m.group(1)
            return self.c[q][m.group(2)][int(m.group(3))]
        m = re.fullmatch(r"(\w+)\[(\d)\]\.v\[(\d)\]", e)      # a[k].v[j]
        if m:
            return self.env[m.group(1)][int(m.group(2))][int(m.group(3))]
        m = re.fullmatch(r"(\w+)(?:\.v)?\[(\d)\]", e)          # a.v[j], m[j], q0[j], a2[j]
        if m:
            return self.env[m.group(1)][int(m.group(2))]
        return self.env[e]                                     # an accumulator

    def asm(self, body, outs, ins):
        outs = re.findall(r'"=&v"\((\w+)\)', outs)
        ins = [self.get(x) for x in re.findall(r'"[vs]"\(([^()]*(?:\([^()]*\))?[^()]*)\)', ins)]
        regs = [None] * len(outs) + ins
        for ln in body.split("\\n\\t"):
            m = re.fullmatch(r"v_mad_u64_u32 %(\d+), vcc, %(\d+), %(\d+), (%\d+|0)", ln)
            if m:
                z = 0 if m.group(4) == "0" else regs[int(m.group(4)[1:])]
                x, y = regs[int(m.group(2))], regs[int(m.group(3))]
                assert x < 1 << 32 and y < 1 << 32
                d = x * y + z
                assert d < 1 << 64, "column accumulator overflow"
                self.max_acc = max(self.max_acc, d)
                regs[int(m.group(1))] = d
                continue
            m = re.fullmatch(r"v_lshrrev_b64 %(\d+), 29, (%\d+)", ln)
            assert m, ln
            regs[int(m.group(1))] = regs[int(m.group(2)[1:])] >> 29
        for i, name in enumerate(outs):
            self.env[name] = regs[i]

    def run(self, body):
        mask = self.c[self.q]["MASK"] if self.q else (1 << 29) - 1
        lines = body.split("\n")
        i = 1   # line 0: the rest of the signature
        while i < len(lines):
            ln = lines[i].strip()
            i += 1
            if not ln or ln.startswith(("uint64_t ", "F29 r1;", "#pragma unroll", "}")):
                continue
            m = re.fullmatch(r"using Q = (\w+);", ln)
            if m:
                self.q = m.group(1)
                mask = self.c[self.q]["MASK"]
                continue
            if re.fullmatch(r"(uint32_t \w+\[9\];\s*)+", ln) or ln.startswith("uint32_t a2[9], c2[9];"):
                for name in re.findall(r"(\w+)\[9\]", ln):
                    self.env[name] = [0] * 9
                continue
            if ln.startswith("for (int i = 0; i < 9; i++) {"):
                for name in ("a", "c"):   # sqr29x2's doubled limbs
                    self.env[name + "2"] = [(x << 1) & 0xFFFFFFFF for x in self.env[name]]
                i += 2
                continue
            if ln.startswith("asm("):
                stmt = [ln]
                while not lines[i - 1].strip().endswith(";"):
                    stmt.append(lines[i].strip())
                    i += 1
                s = " ".join(stmt)
                m = re.fullmatch(r'asm\("(.*?)"\s*: (.*?)\s*: (.*?)\s*: "vcc"\);', s)
                assert m, s
                self.asm(m.group(1), m.group(2), m.group(3))
                continue
            m = re.fullmatch(r"(\w+)\[(\d)\] = \(\(uint32_t\)(\w+) \* (\w+)::INV\) & (\w+)::MASK;", ln)
            if m:
                q = self.q if m.group(4) == "Q" else m.group(4)
                self.env[m.group(1)][int(m.group(2))] = ((self.env[m.group(3)] & 0xFFFFFFFF) *
                                                         self.c[q]["INV"]) & mask
                continue
            m = re.fullmatch(r"(\w+)(?:\.v)?\[(\d)\] = \(uint32_t\)(\w+) & (\w+)::MASK;", ln)
            if m:
                self.env.setdefault(m.group(1), [0] * 9)[int(m.group(2))] = self.env[m.group(3)] & mask
                continue
            m = re.fullmatch(r"(\w+)(?:\.v)?\[8\] = \(uint32_t\)\((\w+) >> 29\);", ln)
            if m:
                self.env.setdefault(m.group(1), [0] * 9)[8] = (self.env[m.group(2)] >> 29) & 0xFFFFFFFF
                continue
            m = re.fullmatch(r"return (\w+);", ln)
            if m:
                return self.env[m.group(1)]
            raise AssertionError(f"emulator: unhandled statement {ln!r}")
        return None


_CACHE = {}


def _emulate(name, q, **inputs):
    if not _CACHE:
        _CACHE["f"], _CACHE["c"] = _functions(_gen()), _consts()
    f = _CACHE["f"]
    emu = _Emu(_CACHE["c"], q)
    for k, v in inputs.items():
        emu.env[k] = v
    ret = emu.run(f[name])
    return ret, emu


def _rand_limbs(rng, bits, top_bits=None):
    lim = int(2 ** bits)
    out = [rng.randrange(lim) for _ in range(8)]
    out.append(rng.randrange(int(2 ** (top_bits if top_bits is not None else bits))))
    return out


def test_generated_montgomery_products_emulated():
    """mul29x2, mul29 (both fields), sqr29x2, mul2sum29 and mulsum29<2..6> as the GPU runs
    them: the result is a b 2^-261 (sums of such) mod the field's prime, with 29-bit low limbs,
    and no column passes 2^64, for normalized operands and for one operand with limbs
    < 2^30.9 (the lazy-normalized inputs of the accumulation), and at all-ones limbs."""
    import random
    rng = random.Random(0xC015)
    inv = {"Fq29": pow(2, -261, _P), "Fr29": pow(2, -261, _R)}
    mod = {"Fq29": _P, "Fr29": _R}
    for trial in range(60):
        wide = 30.9 if trial % 3 else 29
        a, c = _rand_limbs(rng, 29), _rand_limbs(rng, 29)
        b, d = _rand_limbs(rng, wide, 29), _rand_limbs(rng, wide, 29)
        if trial == 0:
            a = b = c = d = [(1 << 29) - 1] * 9
        for q in ("Fq29", "Fr29"):
            _, emu = _emulate("mul29x2_cols", q, a=a, b=b, c=c, d=d)
            r1, r2 = emu.env["r1"], emu.env["r2"]
            assert _val(r1) % mod[q] == _val(a) * _val(b) * inv[q] % mod[q]
            assert _val(r2) % mod[q] == _val(c) * _val(d) * inv[q] % mod[q]
            assert max(r1[:8] + r2[:8]) < 1 << 29
            r, _ = _emulate("mul29_cols", q, a=a, b=b)
            assert _val(r) % mod[q] == _val(a) * _val(b) * inv[q] % mod[q] and max(r[:8]) < 1 << 29
        sa, sc = _rand_limbs(rng, 29.6 if trial % 2 else 29, 29), _rand_limbs(rng, 29, 29)
        _, emu = _emulate("sqr29x2_cols", "Fq29", a=sa, c=sc)
        assert _val(emu.env["r1"]) % _P == _val(sa) ** 2 * inv["Fq29"] % _P
        assert _val(emu.env["r2"]) % _P == _val(sc) ** 2 * inv["Fq29"] % _P
        r, _ = _emulate("mul2sum29_cols", "Fq29", a=a, b=b, c=c, d=d)
        assert _val(r) % _P == (_val(a) * _val(b) + _val(c) * _val(d)) * inv["Fq29"] % _P
        for K in range(2, 7):
            xs = [_rand_limbs(rng, 29) for _ in range(K)]
            ys = [_rand_limbs(rng, 29) for _ in range(K)]
            for q in ("Fq29", "Fr29"):
                r, _ = _emulate(f"mulsum29_cols{K}", q, a=xs, b=ys)
                want = sum(_val(x) * _val(y) for x, y in zip(xs, ys)) * inv[q] % mod[q]
                assert _val(r) % mod[q] == want and max(r[:8]) < 1 << 29


def test_generated_shoup_products_emulated():
    """mul_shoup1 / mul_shoup2 (the NTT twiddles, the grand product's beta products) as the
    GPU runs them: x w mod r + k r with k < 3, normalized, for x < 2^261 with limbs up to
    2^30.6 (f29.h's stated bound) and w < r, ws = floor(w 2^261 / r); no column passes 2^64."""
    import random
    rng = random.Random(0x5A0B)
    for trial in range(80):
        xs, ws, ss = [], [], []
        for _ in range(2):
            x = _rand_limbs(rng, 30.6, 29)
            x[8] = min(x[8], (1 << 29) - 8)                      # x < 2^261
            if trial == 0:
                x = [int(2 ** 30.6)] * 8 + [(1 << 29) - 8]
            w = rng.randrange(_R) if trial else _R - 1
            xs.append(x)
            ws.append(_split(w))
            ss.append(_split((w << 261) // _R))
        r, _ = _emulate("mul_shoup1_cols", None, x0=xs[0], w0=ws[0], s0=ss[0])
        for out, x, w in ((r, xs[0], ws[0]),):
            v = _val(out)
            assert v % _R == _val(x) * _val(w) % _R and v < 3 * _R and max(out) < 1 << 29
        _, emu = _emulate("mul_shoup2_cols", None, x0=xs[0], w0=ws[0], s0=ss[0], x1=xs[1], w1=ws[1], s1=ss[1])
        for out, x, w in ((emu.env["r1"], xs[0], ws[0]), (emu.env["r2"], xs[1], ws[1])):
            v = _val(out)
            assert v % _R == _val(x) * _val(w) % _R and v < 3 * _R and max(out) < 1 << 29
