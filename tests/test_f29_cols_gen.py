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
