"""Generate the committed golden fixtures from the CPU oracle (oracle/plonk.py).

    python tests/golden/make_golden.py

Each case: a seeded synthetic circuit (oracle/synth.py), its snarkjs-0.4 PLONK
zkey (trapdoor tau), the .wtns, and the expected proof for two blinding choices
(all-zero, and SURVEY.md §8d's fixed b_i = SHA-256("nzcb-b"||i) mod r), as binary
(C-ABI layout) and snarkjs JSON. Parity vs snarkjs itself is unpinned.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import binfmt, plonk, synth  # noqa: E402

CASES = [
    # name, power, n_public, n_inputs, seed, tau
    ("p5", 5, 3, 4, 1, 1234567),
    ("p8", 8, 3, 8, 2, 987654321),
]


def blinding_bytes(b):
    return b"".join(x.to_bytes(32, "little") for x in b)


def main():
    for name, power, npub, nin, seed, tau in CASES:
        c = synth.synth_circuit(power, npub, nin, seed=seed)
        zk = plonk.setup(c, tau)
        zbytes = binfmt.write_zkey(zk)
        wbytes = binfmt.write_wtns(c["witness"])
        with open(os.path.join(HERE, f"{name}.zkey"), "wb") as f:
            f.write(zbytes)
        with open(os.path.join(HERE, f"{name}.wtns"), "wb") as f:
            f.write(wbytes)
        meta = {"power": power, "n_public": npub, "n_inputs": nin, "seed": seed, "tau": tau, "proofs": {}}
        for bname, bl in (("zero", None), ("fixed", synth.fixed_blindings())):
            proof, pub = plonk.prove(zk, c["witness"], bl)
            assert plonk.verify_with_trapdoor(zk, pub, proof, tau)
            meta["proofs"][bname] = {
                "blinding": blinding_bytes(bl).hex() if bl else None,
                "proof_bin": plonk.proof_to_bytes(proof).hex(),
                "proof": plonk.proof_to_json_obj(proof),
                "publicSignals": [str(x) for x in pub],
            }
        with open(os.path.join(HERE, f"{name}.json"), "w") as f:
            json.dump(meta, f, indent=1)
        print(name, len(zbytes), "bytes zkey")


if __name__ == "__main__":
    main()
