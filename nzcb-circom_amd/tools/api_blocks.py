#!/usr/bin/env python3
"""Host HIP calls that block inside one proof, from a rocprofv3 --hip-trace --kernel-trace
--marker-trace directory (tools/r4_hiptrace.sh): every API call of the proving thread longer
than --min ms, with its start / end relative to the proof's start and the round it falls in.
  python3 tools/api_blocks.py <trace dir> [--proof K] [--min 0.05]"""
import argparse
import csv
import glob
import os


def rows(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--proof", type=int, default=-2)
    ap.add_argument("--min", type=float, default=0.05)
    a = ap.parse_args()
    ms = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"], r["Thread_Id"])
                for r in rows(a.trace, "*marker_api_trace.csv"))
    proofs = [m for m in ms if m[2] == "plonk_prove"]
    s, e, _, tid = proofs[a.proof]
    rounds = [m for m in ms if s <= m[0] and m[1] <= e and m[2] != "plonk_prove"]
    print("proof %d of %d: %.3f ms (thread %s)" % (a.proof % len(proofs), len(proofs), (e - s) / 1e6, tid))
    for m in rounds:
        print("  %8.3f %8.3f  %s" % ((m[0] - s) / 1e6, (m[1] - s) / 1e6, m[2]))
    api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"])
                 for r in rows(a.trace, "*hip_api_trace.csv") if r["Thread_Id"] == tid)
    tot = {}
    for c in api:
        if not s <= c[0] < e:
            continue
        dur = (c[1] - c[0]) / 1e6
        tot[c[2]] = tot.get(c[2], 0.0) + dur
        if dur >= a.min:
            rnd = next((m[2].split(":")[0] for m in rounds if m[0] <= c[0] < m[1]), "-")
            print("%8.3f %8.3f %7.3f  %-8s %s" % ((c[0] - s) / 1e6, (c[1] - s) / 1e6, dur, rnd, c[2]))
    print("host time in HIP calls by function (ms):")
    for f, t in sorted(tot.items(), key=lambda x: -x[1])[:12]:
        print("  %-40s %8.3f" % (f, t))


if __name__ == "__main__":
    main()
