#!/usr/bin/env python3
"""Isolated MSMs in the Lagrange-basis commitments' regime (round 6): 2^21 + 2 scalars shaped
like nzcp_live gate values (tests/test_gpu_fullsize.py's mix: mostly 0, 1, -1, bytes, short
sums, ~5 % full size), window 17, the sparse schedule (fixed_base = 2) against the dense one
(3); per-phase HIP-event ms (Engine.time_msm_phases).
  python3 tools/sparse_probe.py [--reps 10]"""
import argparse
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import numpy as np
    import nzcb
    r = 21888242871839275222246405745257275088548364400416034343698204186575808495617
    n = (1 << 21) + 2
    rng = random.Random(0x6E7A)
    kinds = rng.choices(range(7), weights=[35, 30, 10, 10, 8, 2, 5], k=n)
    vals = [0 if k == 0 else 1 if k == 1 else r - 1 if k == 2 else rng.randrange(256) if k == 3 else
            rng.randrange(1 << 17) if k == 4 else rng.randrange(1 << 40) if k == 5 else rng.randrange(r)
            for k in kinds]
    raw = b"".join(v.to_bytes(32, "little") for v in vals)
    eng = nzcb.Engine(0, max_log_ntt=-1, max_msm_points=n + 8)
    sc, bases = nzcb.dev_alloc(n * 32), nzcb.dev_alloc(n * 64)
    try:
        eng.random_fr(sc, n, 0x1A6A)
        eng.fixed_base(sc, n, bases)
        nzcb.h2d(sc, raw)
        for mode, name in ((2, "sparse"), (3, "dense17"), (2, "sparse"), (3, "dense17")):
            ph = eng.time_msm_phases(bases, sc, n, False, mode, a.reps)
            print(name, " ".join(f"{k}={v:.4f}" for k, v in ph.items()), flush=True)
    finally:
        nzcb.dev_free(sc)
        nzcb.dev_free(bases)
        eng.close()


if __name__ == "__main__":
    main()
