#!/usr/bin/env python3
"""Kernel microbenchmarks (BASELINE.json configs[1]: BN254 G1 MSM + Fr NTT on one
MI355X, 2^18..2^24). One JSON line per (kernel, size) with HBM-roofline figures:
MSM 96 B/point (64 B affine base + 32 B scalar), NTT 64 B/element/transform
(SURVEY.md §8d). Inputs: pseudo-random Fr scalars, bases [s_i]G1."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nzcb  # noqa: E402

PEAK = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-log", type=int, default=18)
    ap.add_argument("--max-log", type=int, default=24)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    nmax = 1 << args.max_log
    eng = nzcb.Engine(0, max_log_ntt=args.max_log, max_msm_points=nmax)
    sc = nzcb.dev_alloc(nmax * 32)
    out = nzcb.dev_alloc(nmax * 32)
    bases = nzcb.dev_alloc(nmax * 64)
    eng.random_fr(sc, nmax, 0x6E7A6362)
    eng.fixed_base(sc, nmax, bases)
    for lg in range(args.min_log, args.max_log + 1):
        n = 1 << lg
        for inv in (False, True):
            ms = eng.time_ntt(sc, out, lg, inv, args.reps)
            gbs = 64 * n / (ms / 1e3) / 1e9
            print(json.dumps({"kernel": "intt" if inv else "ntt", "log_n": lg, "ms": round(ms, 4),
                              "elements_per_s": round(n / (ms / 1e3), 1), "GBs": round(gbs, 1),
                              "frac": round(gbs / PEAK, 4)}), flush=True)
        for fixed in (False, True):
            ph = eng.time_msm_phases(bases, sc, n, True, fixed, args.reps)
            ms = ph["wall"]
            gbs = 96 * n / (ms / 1e3) / 1e9
            phases = {k: round(v, 4) for k, v in ph.items()
                      if k not in ("wall", "entries", "table_build", "host_enqueue", "host_sort_call")}
            print(json.dumps({"kernel": "msm_fixed_base" if fixed else "msm", "log_n": lg, "ms": round(ms, 4),
                              "phases_ms": phases, "phase_sum_ms": round(sum(phases.values()), 4),
                              "host_enqueue_ms": round(ph.get("host_enqueue", 0), 4),
                              "host_sort_call_ms": round(ph.get("host_sort_call", 0), 4),
                              "table_build_ms": round(ph.get("table_build", 0), 2), "entries": int(ph.get("entries", 0)),
                              "points_per_s": round(n / (ms / 1e3), 1), "GBs": round(gbs, 1),
                              "frac": round(gbs / PEAK, 5)}), flush=True)
    for p in (sc, out, bases):
        nzcb.dev_free(p)


if __name__ == "__main__":
    main()
