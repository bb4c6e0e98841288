"""Witness programs re-indexed to another wire order by signal name (VERDICT r2 item 7,
SURVEY.md §8f row f3): nzcb/circuit.py writes a circom-style .sym for every signal
(hierarchical main.<component>.<signal> names following the circom templates,
nzcb/nzcpgen.py), and nzcb_wprog_remap (csrc/wvm.hip) maps the program onto any .sym's
order, e.g. circom's own nzcp_live.sym for the reference's nzcp_live_final.zkey
(/root/reference/README.md:43). Checked here against a permuted self-generated .sym, on
the CPU (the library's remap, the oracle's evaluation of the remapped program); the GPU
run of a remapped program and a proof over a permuted r1cs are in tests/test_gpu_wvm.py.
The names are those the reference's templates declare (tests/test_circom_names.py); which of
two equal signals circom keeps as the wire (the other listed with -1) is unpinned: circom
and its output are not on disk."""
import random

import pytest

import nzcb
from nzcb import circuit, nzcpgen
from oracle import wvm

R = circuit.R


def permuted_sym(c, seed):
    """The circuit's .sym with wires 1.. shuffled (outputs and inputs included) and some
    extra optimized-out (-1) names, as circom writes for substituted signals."""
    perm = list(range(1, c.n_wires))
    random.Random(seed).shuffle(perm)
    new = {old: i + 1 for i, old in enumerate(perm)}
    lines = [f"{k + 1},{new[wire]},0,{c.names[wire]}" for k, wire in enumerate(sorted(c.names))]
    lines += [f"{len(lines) + 1},-1,0,main.optimizedAway[{i}]" for i in range(3)]
    random.Random(seed + 1).shuffle(lines)
    return ("\n".join(lines) + "\n").encode(), new


def test_sym_names_every_wire_once():
    c = nzcpgen.wrapper_circuit("readMapLength_test")
    sym = c.write_sym().decode().splitlines()
    wires = [int(x.split(",")[1]) for x in sym]
    names = [x.split(",", 3)[3] for x in sym]
    # the wires in order, then the further names (signals sharing a wire, or -1)
    assert wires[:c.n_wires - 1] == list(range(1, c.n_wires)) and len(set(names)) == len(names)
    assert all(0 < x < c.n_wires or x == -1 for x in wires[c.n_wires - 1:])
    assert names[:2] == ["main.len", "main.nextPos"] and names[2] == "main.pos"     # circom's main order
    assert names[3:10] == [f"main.bytes[{i}]" for i in range(7)]


def test_nzcp_live_sym_follows_the_templates():
    c = nzcpgen.nzcp_pub_identity(**nzcpgen.LIVE)
    names = set(c.names.values())
    assert len(names) == c.n_wires - 1
    for want in ("main.out[0]", "main.toBeSigned[0]", "main.toBeSignedLen", "main.data[159]",
                 "main.lteMaxToBeSignedBytes.n2b.out[0]", "main.ltLen[350].n2b.out[9]", "main.ToBeSigned[350]",
                 "main.n2bNullifier[63].out[7]", "main.n2bExp.out[31]"):
        assert want in names, want
    for prefix in ("main.tbsSha256.", "main.readMapLengthClaims.", "main.findVC.", "main.readCredSubj.",
                   "main.nullifier.", "main.nullifierSha512."):
        assert any(n.startswith(prefix) for n in names), prefix


@pytest.mark.parametrize("name,inputs", [
    ("readMapLength_test", [0, 0xA2, 4, 5, 5, 4, 0, 0]),
    ("skipValue5_test", [0x83, 0x61, 0x71, 0x17, 0x17, 0]),
    ("copyString_test", [0x62, 0x61, 0x62, 0, 0, 0])])
def test_remap_permutes_the_witness(name, inputs):
    c = nzcpgen.wrapper_circuit(name)
    prog = c.write_program()
    sym, new = permuted_sym(c, 7)
    mapped = nzcb.wprog_remap(prog, c.write_sym(), sym)
    base, fail = wvm.evaluate(prog, inputs)
    got, fail2 = wvm.evaluate(mapped, inputs)
    assert fail is None and fail2 is None
    assert got[0] == 1 and len(got) == c.n_wires
    assert all(got[new[k]] == base[k] for k in range(1, c.n_wires))
    # the permuted witness satisfies the permuted r1cs
    for A, B, Cc in c.constraints:
        ev = lambda x: sum(v * got[new[i]] if i else v for i, v in x.items()) % R   # noqa: E731
        assert (ev(A) * ev(B) - ev(Cc)) % R == 0


def test_remap_reports_unmatched_signals():
    c = nzcpgen.wrapper_circuit("readMapLength_test")
    sym, _ = permuted_sym(c, 3)
    broken = sym.replace(b"main.nextPos", b"main.somethingElse")
    with pytest.raises(nzcb.NzcbError) as e:
        nzcb.wprog_remap(c.write_program(), c.write_sym(), broken)
    assert e.value.unmatched == 1 and "main.somethingElse" in str(e.value)
    mapped = nzcb.wprog_remap(c.write_program(), c.write_sym(), sym)
    with pytest.raises(nzcb.NzcbError, match="already remapped"):
        nzcb.wprog_remap(mapped, c.write_sym(), sym)


def test_remap_subset_target():
    """A target that names fewer signals than the program (circom --O2 drops substituted
    ones): the remapped witness has the target's size and the program keeps computing its
    own intermediates in scratch."""
    c = nzcpgen.wrapper_circuit("quinSelector3_test")
    prog = c.write_program()
    keep = [w for w in sorted(c.names) if not c.names[w].startswith("main.eqs")]
    sym = "".join(f"{k + 1},{k + 1},0,{c.names[w]}\n" for k, w in enumerate(keep)).encode()
    mapped = nzcb.wprog_remap(prog, c.write_sym(), sym)
    base, _ = wvm.evaluate(prog, [1, 2, 3, 2])
    got, _ = wvm.evaluate(mapped, [1, 2, 3, 2])
    assert len(got) == len(keep) + 1 and got[1:] == [base[w] for w in keep]


def test_write_artifacts(tmp_path):
    """nzcplive.write_artifacts: r1cs, program and its .sym for a circuit, consistent with
    each other (the remap of the program onto its own .sym is the identity)."""
    from nzcb import nzcplive
    from oracle import r1cs as r1
    out = nzcplive.write_artifacts(str(tmp_path), params=dict(nzcpgen.EXAMPLE), name="nzcp_example")
    prog, sym = open(out["program"], "rb").read(), open(out["sym"], "rb").read()
    rd = r1.read_r1cs(open(out["r1cs"], "rb").read())
    wires = {int(x.split(b",")[1]) for x in sym.splitlines()}
    assert rd["nWires"] == wvm.parse(prog)["n_wires"] == max(wires) + 1
    assert wires == set(range(1, rd["nWires"])) | {-1}     # every wire named; substituted signals -1
    same = nzcb.wprog_remap(prog, sym, sym)
    assert wvm.parse(same)["wmap"] == list(range(rd["nWires"]))
