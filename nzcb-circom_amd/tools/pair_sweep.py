#!/usr/bin/env python3
"""Fixed-base MSM at 2^lg points with 0..R batch-affine pairing rounds (msm.hip
msm_pair29_kernel): per-phase HIP-event times, and the results of every round count
must agree (the schedule changes, the group element does not)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nzcb  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log", type=int, default=21)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    n = 1 << args.log
    eng = nzcb.Engine(0, max_log_ntt=-1, max_msm_points=n + 8)
    sc = nzcb.dev_alloc(n * 32)
    bases = nzcb.dev_alloc(n * 64)
    eng.random_fr(sc, n, 0x6E7A6362)
    eng.fixed_base(sc, n, bases)
    eng.random_fr(sc, n, 0x5EED)
    ref = None
    try:
        for r in range(args.rounds + 1):
            nzcb.msm_set_pair_rounds(r)
            got = eng.msm_fixed_dev(bases, n, sc, n, True)
            ref = ref or got
            ph = eng.time_msm_phases(bases, sc, n, True, True, args.reps)
            print(json.dumps({"log_n": args.log, "pair_rounds": r, "agrees": got == ref,
                              "ms": round(ph["wall"], 4),
                              "phases_ms": {k: round(v, 4) for k, v in ph.items() if k != "wall"}}), flush=True)
    finally:
        nzcb.msm_set_pair_rounds(-1)
        nzcb.dev_free(sc)
        nzcb.dev_free(bases)
        eng.close()


if __name__ == "__main__":
    main()
