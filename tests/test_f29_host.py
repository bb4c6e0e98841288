"""csrc/f29.h's 9x29-bit primitives built for the host (tests/native/f29_host.cpp, clang++
from the ROCm toolchain; f29.h is header-only and host-compilable) against exact integers:
the Shoup twiddle product of the NTT (single and paired), the low-half product that builds
the twiddles' Shoup quotients, and the Montgomery product. Catches an indexing slip in the
C++ that the integer restatement (tests/test_shoup_math.py) cannot."""
import os
import random
import shutil
import subprocess

import pytest

from oracle.bn254 import R_MOD as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CXX = shutil.which("clang++") or "/opt/rocm/lib/llvm/bin/clang++"
M = (1 << 29) - 1
NINV = (-pow(R, -1, 1 << 261)) % (1 << 261)


def limbs(x):
    return [(x >> (29 * i)) & M for i in range(9)]


def val(l):
    return sum(v << (29 * i) for i, v in enumerate(l))


def hexl(l):
    return " ".join("%x" % v for v in l)


@pytest.fixture(scope="module")
def host_bin(tmp_path_factory):
    if not os.path.exists(CXX):
        pytest.skip("no clang++")
    out = str(tmp_path_factory.mktemp("f29") / "f29_host")
    subprocess.run([CXX, "-O1", "-std=c++17", os.path.join(ROOT, "tests", "native", "f29_host.cpp"), "-o", out],
                   check=True)
    return out


def _run(binary, lines):
    p = subprocess.run([binary], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    return [[int(t, 16) for t in ln.split()] for ln in p.stdout.splitlines()]


def _wide(X, rng):
    xl = limbs(X)
    for i in range(8, 0, -1):
        if xl[i] and rng.random() < 0.5:
            b = rng.randrange(0, min(xl[i], 3) + 1)
            xl[i] -= b
            xl[i - 1] += b << 29
    if max(xl) >= int(2 ** 30.7):
        xl = limbs(X)
    return xl


def test_shoup_products_host(host_bin):
    rng = random.Random(0xF29)
    lines, want = [], []
    for it in range(400):
        W, X = rng.randrange(R), rng.randrange(99 * R)
        ws = (W << 261) // R
        xl = _wide(X, rng)
        if it % 2:
            W2, X2 = rng.randrange(R), rng.randrange(99 * R)
            lines.append("2 " + " ".join(hexl(v) for v in (xl, limbs(W), limbs(ws), _wide(X2, rng), limbs(W2),
                                                           limbs((W2 << 261) // R))))
            want += [(X * W) % R, (X2 * W2) % R]
        else:
            lines.append("1 " + " ".join(hexl(v) for v in (xl, limbs(W), limbs(ws))))
            want.append((X * W) % R)
    got = _run(host_bin, lines)
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert all(v <= M for v in g)
        assert val(g) % R == w and val(g) < 3 * R


def test_lo261_and_mont_host(host_bin):
    rng = random.Random(0x261)
    lines, want = [], []
    for _ in range(200):
        m = rng.randrange(R)
        lines.append("3 " + hexl(limbs(m)) + " " + hexl(limbs(NINV)))
        want.append(("lo", (m * NINV) % (1 << 261)))
        a, b = rng.randrange(R), rng.randrange(R)
        lines.append("4 " + hexl(limbs(a)) + " " + hexl(limbs(b)))
        want.append(("mont", (a * b * pow(2, -261, R)) % R))
    got = _run(host_bin, lines)
    for g, (kind, w) in zip(got, want):
        if kind == "lo":
            assert val(g) == w
        else:
            assert val(g) % R == w and val(g) < 2 * R


def test_exponent_261_conversions_host(host_bin):
    """The grand product's radix change (prover.hip k_perm_tile): fr_to261 shifts a
    Montgomery-256 value's limbs by 5 bits (x 32, normalized), fr_from261 returns an
    exponent-261 value to canonical Montgomery-256."""
    rng = random.Random(0x261261)
    xs = [0, 1, R - 1, (1 << 253) + 12345] + [rng.randrange(R) for _ in range(200)]
    lines = ["5 " + " ".join("%x" % ((x >> (32 * i)) & 0xFFFFFFFF) for i in range(8)) for x in xs]
    ys = [rng.randrange(4 * R) for _ in range(200)]
    lines += ["6 " + hexl(limbs(y)) for y in ys]
    got = _run(host_bin, lines)
    for g, x in zip(got[:len(xs)], xs):
        assert all(v <= M for v in g) and val(g) == 32 * x
    for g, y in zip(got[len(xs):], ys):
        z = sum(v << (32 * i) for i, v in enumerate(g))
        assert z < R and z == (y * pow(2, -5, R)) % R       # exponent 261 -> 256: y 2^-5
