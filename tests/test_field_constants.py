"""The modulus constants the HIP kernels are compiled with (csrc/field.h, csrc/f29.h)
against the BN254 values of the oracle: limbs, Montgomery inverses, R mod p, R^2 mod p,
and the borrowed-limb multiples k*p that the 9x29-bit subtraction relies on (every limb
>= 2^29 - 1, so a normalized subtrahend never drives a limb negative)."""
import os
import re

import pytest

from oracle.bn254 import P_MOD, R_MOD

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "nzcb-circom_amd", "csrc")


def _struct_consts(path, struct):
    src = open(os.path.join(CSRC, path)).read()
    body = re.search(r"struct %s \{(.*?)\n\};" % struct, src, re.S).group(1)
    out = {}
    for m in re.finditer(r"static constexpr uint(?:32|64)_t (\w+)(?:\[(\d+)\])? = ([^;]+);", body):
        vals = [int(v.rstrip("uUlL"), 16) for v in re.findall(r"0x[0-9a-fA-F]+[uUlL]*", m.group(3))]
        if vals:  # skip expressions such as MASK = (1u << 29) - 1
            out[m.group(1)] = vals if m.group(2) else vals[0]
    return out


def _val(limbs, bits):
    return sum(v << (bits * i) for i, v in enumerate(limbs))


@pytest.mark.parametrize("struct,mod", [("FqParams", P_MOD), ("FrParams", R_MOD)])
def test_field_h_params(struct, mod):
    c = _struct_consts("field.h", struct)
    assert _val(c["P"], 32) == mod
    assert (c["INV"] * mod) % (1 << 32) == (1 << 32) - 1          # -p^-1 mod 2^32
    assert (c["INV64"] * mod) % (1 << 64) == (1 << 64) - 1
    assert _val(c["ONE"], 32) == (1 << 256) % mod
    assert _val(c["R2"], 32) == (1 << 512) % mod


@pytest.mark.parametrize("struct,mod,ks", [("Fq29", P_MOD, {"K2": 2, "K4": 4, "K6": 6, "K8": 8}),
                                           ("Fr29", R_MOD, {"K2": 2, "K4": 4})])
def test_f29_params(struct, mod, ks):
    c = _struct_consts("f29.h", struct)
    assert _val(c["P"], 29) == mod and all(v < (1 << 29) for v in c["P"])
    assert (c["INV"] * mod) % (1 << 29) == (1 << 29) - 1          # -p^-1 mod 2^29
    for name, k in ks.items():
        limbs = c[name]
        assert _val(limbs, 29) == k * mod, name
        assert all(v >= (1 << 29) - 1 for v in limbs[:8]), name     # borrowed form
        assert all(v < (1 << 32) - (1 << 30) for v in limbs), name   # a + K - b fits 32 bits
    if "ONE" in c:
        assert _val(c["ONE"], 29) == (1 << 261) % mod
    if "C256" in c:
        assert _val(c["C256"], 29) == (1 << 256) % mod


def test_fr29_shoup_constants():
    """The NTT's Shoup products (f29.h mul_shoup, round 5): RP = 2^261 - r, NINV = -r^-1 mod
    2^261, both as 9 normalized 29-bit limbs."""
    c = _struct_consts("f29.h", "Fr29")
    assert _val(c["RP"], 29) == (1 << 261) - R_MOD and all(v < (1 << 29) for v in c["RP"])
    assert (_val(c["NINV"], 29) * R_MOD) % (1 << 261) == (1 << 261) - 1
    assert all(v < (1 << 29) for v in c["NINV"])
