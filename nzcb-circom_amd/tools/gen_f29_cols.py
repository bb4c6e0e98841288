#!/usr/bin/env python3
"""Generates csrc/f29_cols.h: the device bodies of csrc/f29.h's 9x29 products (mul29,
mul29x2, sqr29x2, mul2sum29, mulsum29<K>, the Shoup pair and single) with one inline-asm statement per
product column.

The compiler puts an s_nop after every inline-asm statement; with one statement per mad
pair (f29.h mad29x2) the bucket accumulation carried 1,646 of them per loop body against
2,506 v_mad_u64_u32. Here a statement holds a whole column of both chains: the previous
column's m_i * P_0 pair and carry shift, then every product term of the column, so a
product pair pays 17 of them. The Montgomery quotient digits m_i and the result limbs
(low 32 bits of an accumulator) stay C between the statements.

    python3 tools/gen_f29_cols.py > csrc/f29_cols.h
"""


class Blk:
    """One asm statement. Outputs: each chain's new accumulator value (operands 0..k-1,
    early-clobber). Inputs: each chain's previous value (unless it starts at 0), then the
    multiplicands. The first instruction of a chain reads the previous value and writes
    the new one (v_mad_u64_u32 and v_lshrrev_b64 are three-address), so the previous value
    stays readable after the statement: the C extraction of its low limb needs no copy."""

    def __init__(self, olds, news):
        self.olds, self.news = olds, news  # per chain: previous value (None: starts at 0), new value
        self.k = len(news)
        self.ins = [("v", o) for o in olds if o is not None]
        self.lines = []
        self.started = set()

    def op(self, cons, expr):
        key = (cons, expr)
        if key not in self.ins:
            self.ins.append(key)
        return "%" + str(self.k + self.ins.index(key))

    def _src(self, c):
        if c in self.started:
            return f"%{c}"
        self.started.add(c)
        return "0" if self.olds[c] is None else self.op("v", self.olds[c])

    def mad(self, c, x, y, ycons="v"):
        xo, yo = self.op("v", x), self.op(ycons, y)
        self.lines.append(f"v_mad_u64_u32 %{c}, vcc, {xo}, {yo}, {self._src(c)}")

    def shift(self, c):
        self.lines.append(f"v_lshrrev_b64 %{c}, 29, {self._src(c)}")

    def emit(self, ind="  "):
        assert self.lines and len(self.started) == self.k
        outs = ", ".join(f'"=&v"({a})' for a in self.news)
        ins = ", ".join(f'"{c}"({e})' for c, e in self.ins)
        body = "\\n\\t".join(self.lines)
        return [f'{ind}asm("{body}"', f"{ind}    : {outs}", f"{ind}    : {ins}", f'{ind}    : "vcc");']


class Chains:
    """Accumulator values, one C variable per statement and chain (acc0, acc1, ...)."""

    def __init__(self, names):
        self.names, self.cur, self.n, self.decl = names, [None] * len(names), 0, []

    def block(self):
        news = [f"{nm}{self.n}" for nm in self.names]
        self.decl += news
        b = Blk(list(self.cur), news)
        self.cur = news
        self.n += 1
        return b


def write_product(name, sig, pairs, sq=None, Q="Q", template="template <class Q>", pre=()):
    """pairs: per chain, a function i -> list of (x, y) product terms of column i."""
    k = len(pairs)
    ch = Chains(["acc", "bcc", "ccc"][:k])
    ms = ["m", "n", "o"][:k]
    body = []
    carry = []  # what the next statement starts with: previous m_i P_0 and/or shifts
    for i in range(17):
        b = ch.block()
        for kind, c, extra in carry:
            if kind == "mp0":
                b.mad(c, f"{ms[c]}[{extra}]", f"{Q}::P[0]", "s")
            else:
                b.shift(c)
        tl = [p(i) for p in pairs]
        for t in range(max(len(x) for x in tl)):
            for c in range(k):
                if t < len(tl[c]):
                    b.mad(c, *tl[c][t])
        jr = range(0, i) if i < 9 else range(i - 8, 9)
        for j in jr:
            for c in range(k):
                b.mad(c, f"{ms[c]}[{j}]", f"{Q}::P[{i - j}]", "s")
        body += b.emit()
        if i < 9:
            for c in range(k):
                body.append(f"  {ms[c]}[{i}] = ((uint32_t){ch.cur[c]} * {Q}::INV) & {Q}::MASK;")
            carry = [("mp0", c, i) for c in range(k)] + [("sh", c, None) for c in range(k)]
        else:
            for c in range(k):
                body.append(f"  r{c + 1}.v[{i - 9}] = (uint32_t){ch.cur[c]} & {Q}::MASK;")
            carry = [("sh", c, None) for c in range(k)]
    for c in range(k):  # the top limb: the last column's carry
        body.append(f"  r{c + 1}.v[8] = (uint32_t)({ch.cur[c]} >> 29);")
    out = [template] if template else []
    out.append(f"__device__ __forceinline__ {sig} {{")
    out += ["  " + p for p in pre]
    out.append("  " + " ".join(f"uint32_t {m}[9];" for m in ms))
    out.append("  uint64_t " + ", ".join(ch.decl) + ";")
    return out + body


def write_shoup(k):
    """mul_shoup_n<k> (f29.h), k = 1 or 2: q from columns 7..16 of x ws, then
    x w + q (2^261 - r) over columns 0..8, the k products side by side."""
    xs, ws, ss, qs = ["x0", "x1"][:k], ["w0", "w1"][:k], ["s0", "s1"][:k], ["q0", "q1"][:k]
    T = range(k)
    ch = Chains(["acc", "bcc"][:k])
    body = []
    pend_shift = False
    for c in range(7, 17):
        b = ch.block()
        if pend_shift:
            for t in T:
                b.shift(t)
        for j in range(max(0, c - 8), min(c, 8) + 1):
            for t in T:
                b.mad(t, f"{xs[t]}.v[{j}]", f"{ss[t]}.v[{c - j}]")
        if c < 9:
            for t in T:
                b.shift(t)
            pend_shift = False
        else:
            pend_shift = True
        body += b.emit()
        if c >= 9:
            for t in T:
                body.append(f"  {qs[t]}[{c - 9}] = (uint32_t){ch.cur[t]} & Q::MASK;")
    for t in T:
        body.append(f"  {qs[t]}[8] = (uint32_t)({ch.cur[t]} >> 29);")
    ch.cur = [None] * k  # the second product starts at 0
    pend_shift = False
    for c in range(9):
        b = ch.block()
        if pend_shift:
            for t in T:
                b.shift(t)
        for j in range(c + 1):
            for t in T:
                b.mad(t, f"{xs[t]}.v[{j}]", f"{ws[t]}.v[{c - j}]")
            for t in T:
                b.mad(t, f"{qs[t]}[{j}]", f"Q::RP[{c - j}]", "s")
        body += b.emit()
        for t in T:
            body.append(f"  r{t + 1}.v[{c}] = (uint32_t){ch.cur[t]} & Q::MASK;")
        pend_shift = True
    if k == 2:
        out = ["__device__ __forceinline__ void mul_shoup2_cols(const F29& x0, const F29& w0, const F29& s0, "
               "const F29& x1, const F29& w1, const F29& s1, F29& r1, F29& r2) {"]
    else:
        out = ["__device__ __forceinline__ F29 mul_shoup1_cols(const F29& x0, const F29& w0, const F29& s0) {",
               "  F29 r1;"]
    out += ["  using Q = Fr29;",
            "  " + " ".join(f"uint32_t {q}[9];" for q in qs),
            "  uint64_t " + ", ".join(ch.decl) + ";"]
    return out + body + (["  return r1;"] if k == 1 else []) + ["}"]


def main():
    L = ["// GENERATED by tools/gen_f29_cols.py from the column schedules of csrc/f29.h's",
         "// mul29x2 / sqr29x2 / mul2sum29 / mul_shoup_n<2> / mul_shoup_n<1> / mul29 / mulsum29 -- do not edit. One inline-asm statement per product",
         "// column (see the generator's docstring); included by f29.h for the device compile.",
         "#pragma once", ""]
    mul = lambda a, b: (lambda i: [(f"{a}.v[{j}]", f"{b}.v[{i - j}]")
                                   for j in range(max(0, i - 8), min(i, 8) + 1)])
    L += write_product("mul29x2_cols", "void mul29x2_cols(const F29& a, const F29& b, const F29& c, const F29& d, "
                       "F29& r1, F29& r2)", [mul("a", "b"), mul("c", "d")])
    L.append("}")
    L.append("")

    def sq(a, a2):
        def t(i):
            r = [(f"{a}.v[{j}]", f"{a2}[{i - j}]") for j in range(max(0, i - 8), 9) if 2 * j < i]
            if i % 2 == 0 and i // 2 <= 8:
                r.append((f"{a}.v[{i // 2}]", f"{a}.v[{i // 2}]"))
            return r
        return t
    L += write_product("sqr29x2_cols", "void sqr29x2_cols(const F29& a, const F29& c, F29& r1, F29& r2)",
                       [sq("a", "a2"), sq("c", "c2")], Q="Fq29", template=None,
                       pre=["uint32_t a2[9], c2[9];",
                            "#pragma unroll",
                            "for (int i = 0; i < 9; i++) {",
                            "  a2[i] = a.v[i] << 1;",
                            "  c2[i] = c.v[i] << 1;",
                            "}"])
    L.append("}")
    L.append("")

    def two(i):
        r = []
        for j in range(max(0, i - 8), min(i, 8) + 1):
            r += [(f"a.v[{j}]", f"b.v[{i - j}]"), (f"c.v[{j}]", f"d.v[{i - j}]")]
        return r
    body = write_product("mul2sum29_cols", "F29 mul2sum29_cols(const F29& a, const F29& b, const F29& c, const F29& d)",
                         [two], Q="Fq29", template=None)
    body.insert(body.index("  uint32_t m[9];") + 1, "  F29 r1;")
    L += body
    L.append("  return r1;")
    L.append("}")
    L.append("")
    body = write_product("mul29_cols", "F29 mul29_cols(const F29& a, const F29& b)", [mul("a", "b")])
    body.insert(body.index("  uint32_t m[9];") + 1, "  F29 r1;")
    L += body
    L.append("  return r1;")
    L.append("}")
    L.append("")
    L += write_shoup(2)
    L.append("")
    L += write_shoup(1)
    L.append("")
    for K in range(2, 7):  # mulsum29<Q, K> (sum of K products, one reduction)
        def terms(i, K=K):
            r = []
            js = range(0, i + 1) if i < 9 else range(i - 8, 9)
            for j in js:
                r += [(f"a[{k}].v[{j}]", f"b[{k}].v[{i - j}]") for k in range(K)]
            return r
        body = write_product(f"mulsum29_cols{K}", f"F29 mulsum29_cols{K}(const F29 (&a)[{K}], const F29 (&b)[{K}])",
                             [terms])
        body.insert(body.index("  uint32_t m[9];") + 1, "  F29 r1;")
        L += body
        L.append("  return r1;")
        L.append("}")
        L.append("")
    print("\n".join(L))


if __name__ == "__main__":
    main()
