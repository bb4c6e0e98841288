#!/usr/bin/env python3
"""The fixed-base MSM alone (bench.py accumulate_probe's workload: 2^21 + 6 points,
c = 17 table) for PMC passes: rocprofv3 --pmc <counters> -- python3 tools/acc_probe.py"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nzcb  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log", type=int, default=21)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    n = (1 << a.log) + 6
    eng = nzcb.Engine(0, max_log_ntt=-1, max_msm_points=n + 8)
    sc, bases = nzcb.dev_alloc(n * 32), nzcb.dev_alloc(n * 64)
    eng.random_fr(sc, n, 0x70726F6265)
    eng.fixed_base(sc, n, bases)
    eng.random_fr(sc, n, 0x5CA1A25)
    eng.time_msm_phases(bases, sc, n, True, True, 1)
    ph = eng.time_msm_phases(bases, sc, n, True, True, a.reps)
    print(json.dumps({k: round(v, 4) for k, v in ph.items()}))
    nzcb.dev_free(sc)
    nzcb.dev_free(bases)
    eng.close()


if __name__ == "__main__":
    main()
