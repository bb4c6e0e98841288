"""circom name parity of the .sym: every signal
the reference's own templates declare (NZCPPubIdentity, FindCWTClaims, ReadCredSubj,
ConstructNullifier, the cbortpl templates, QuinSelector; extracted from
/root/reference/circuits/*.circom by tests/golden/make_circom_names.py into
tests/golden/circom_names.json) appears in nzcb/circuit.py write_sym() of nzcp_live under
circom's hierarchical name main.<component>[i].<signal>[j], with every array expanded to the
shapes nzcp_live's main NZCPPubIdentity(1, 351, 0, 4, 2, 4) gives it (/root/reference/
circuits/nzcp_live.circom). Signals that circom would substitute away are in the .sym too,
with wire -1, as circom writes them.

Templates from libraries the reference downloads at build time (circomlib's LessThan,
IsZero, IsEqual, Num2Bits, Bits2Num, ShR; CalculateTotal; Sha256Var; Sha512) are not on
disk: their internals stay parity unpinned, and only their instance names are checked
(each instance owns at least one named signal)."""
import json
import os
import re

import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "circom_names.json")
MAIN = ("NZCPPubIdentity", [1, 351, 0, 4, 2, 4])   # /root/reference/circuits/nzcp_live.circom


def log2(x):  # /root/reference/circuits/log2.circom
    z = -1
    while x:
        z += 1
        x //= 2
    return z


def pow_(x, y):  # /root/reference/circuits/pow.circom
    return 1 if y == 0 else x * pow_(x, y - 1)


def ev(expr: str, env: dict):
    """A circom expression of template parameters and vars, as Python: `\\` is integer
    division, `a ? b : c` a conditional (one level)."""
    e = expr.replace("\\", "//")
    m = re.fullmatch(r"(.+?)\?(.+?):(.+)", e)
    if m:
        e = f"(({m.group(2)}) if ({m.group(1)}) else ({m.group(3)}))"
    return eval(e, {"log2": log2, "pow": pow_}, dict(env))  # noqa: S307 (extracted shape expressions)


def indices(shape):
    if not shape:
        yield ""
        return
    for i in range(shape[0]):
        for rest in indices(shape[1:]):
            yield f"[{i}]{rest}"


def expected(tmpls, name, args, path, names, externals):
    t = tmpls[name]
    env = dict(zip(t["params"], args))
    for var, expr in t["vars"]:
        try:
            env[var] = ev(expr, env)
        except Exception:  # loop-header vars and the like: not used by shapes
            pass
    for sig, _kind, dims in t["signals"]:
        for idx in indices([ev(d, env) for d in dims]):
            names.append(f"{path}.{sig}{idx}")
    for comp, dims, sub, argtext in t["components"]:
        if sub is None:  # declared, never instantiated: no signals (FindCWTClaims.decodeUintValue)
            continue
        for idx in indices([ev(d, env) for d in dims]):
            inst = f"{path}.{comp}{idx}"
            if sub in tmpls:
                sub_args = [ev(a, env) for a in re.split(r",(?![^\[]*\])", argtext)] if argtext else []
                expected(tmpls, sub, sub_args, inst, names, externals)
            else:
                externals.append((inst, sub))


@pytest.fixture(scope="module")
def live_sym():
    from nzcb import nzcpgen
    c = nzcpgen.nzcp_pub_identity(**nzcpgen.LIVE)
    lines = c.write_sym().decode().splitlines()
    return {x.split(",", 3)[3]: int(x.split(",", 3)[1]) for x in lines}


@pytest.fixture(scope="module")
def reference_names():
    tmpls = json.load(open(GOLD))["templates"]
    names, externals = [], []
    expected(tmpls, MAIN[0], MAIN[1], "main", names, externals)
    return names, externals


def test_golden_extraction_covers_the_reference_templates():
    tmpls = json.load(open(GOLD))["templates"]
    assert {"NZCPPubIdentity", "FindCWTClaims", "FindCredSubj", "ReadCredSubj", "ConstructNullifier", "GetType",
            "GetX", "GetV", "DecodeUint23", "DecodeUint", "ReadType", "SkipValueScalar", "SkipValue", "StringEquals",
            "ReadStringLength", "ReadMapLength", "CopyString", "QuinSelector"} <= set(tmpls)
    top = tmpls["NZCPPubIdentity"]
    assert [s[0] for s in top["signals"]] == ["toBeSigned", "toBeSignedLen", "data", "out", "ToBeSigned", "exp",
                                             "nullifierBits"]


def test_every_reference_signal_is_named(live_sym, reference_names):
    names, _ = reference_names
    assert len(names) > 100000
    missing = [n for n in names if n not in live_sym]
    assert not missing, f"{len(missing)} of {len(names)} missing, e.g. {missing[:10]}"


def test_every_library_instance_is_named(live_sym, reference_names):
    """circomlib / sha256-var / sha512 instances (internals unpinned): the instance exists."""
    _, externals = reference_names
    prefixes = set()
    for n in live_sym:
        parts = n.split(".")
        for k in range(2, len(parts)):
            prefixes.add(".".join(parts[:k]))
    missing = [(p, t) for p, t in externals if p not in prefixes]
    assert not missing, f"{len(missing)} of {len(externals)} instances missing, e.g. {missing[:10]}"


def test_io_and_substituted_signals_wires(live_sym):
    """main's outputs and inputs keep circom's wires 1..; a signal equal to another signal
    (a component's input, an output passed on) shares that signal's wire, and one that is a
    constant or a combination of several wires (circom --O2 substitutes it) is listed
    with -1, as circom writes it."""
    assert live_sym["main.out[0]"] == 1 and live_sym["main.out[2]"] == 3
    assert live_sym["main.toBeSigned[0]"] == 4 and live_sym["main.data[159]"] == 4 + 2808 + 160
    # nullifierBits: the SHA-512 gadget's output bits, one wire each
    assert live_sym["main.nullifierBits[0]"] > 0
    # an alias: the first map-length read's byte array is main's ToBeSigned
    assert live_sym["main.readMapLengthClaims.bytes[7]"] == live_sym["main.ToBeSigned[7]"]
    assert live_sym["main.findVC.decodeUint[0].getV_24.quinSelector.in[3]"] == live_sym["main.ToBeSigned[3]"]
    # combinations and constants: Bits2Num's sum, a padded name byte, QuinSelector(0)'s out
    assert live_sym["main.b2n[0].out"] == -1
    assert live_sym["main.readCredSubj.givenName[63]"] == -1
    assert live_sym["main.findVC.skipValue[0].qs.out"] == -1


def test_sym_names_are_unique_and_cover_every_wire(live_sym):
    from nzcb import nzcpgen
    c = nzcpgen.nzcp_pub_identity(**nzcpgen.LIVE)
    lines = c.write_sym().decode().splitlines()
    assert len(lines) == len(live_sym)            # no name twice
    wires = {int(x.split(",")[1]) for x in lines}
    assert set(range(1, c.n_wires)) <= wires and wires - set(range(1, c.n_wires)) == {-1}
