#!/usr/bin/env python3
"""One proof's kernel timeline from a rocprofv3 --kernel-trace --marker-trace directory
(bench.py --lanes 1): the round ranges, then every kernel that starts inside the proof with
start / end / duration (ms from the proof's start) and its stream / hardware queue, and the
GPU-idle gaps longer than --gap ms. DESIGN.md §Concurrency reads the round-4 changes off it.
  python3 tools/timeline.py <trace dir> [--proof K] [--gap 0.15]"""
import argparse
import csv
import glob
import os


def load(d):
    kf = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    mf = glob.glob(os.path.join(d, "**", "*marker_api_trace.csv"), recursive=True)[0]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r["Kernel_Name"].split("(")[0].replace("void ", "").replace("nzcb::", ""),
                 "%s/%s" % (r["Stream_Id"], r["Queue_Id"])) for r in csv.DictReader(open(kf)))
    ms = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"])
                for r in csv.DictReader(open(mf)))
    return ks, ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--proof", type=int, default=-1, help="index among the plonk_prove ranges")
    ap.add_argument("--gap", type=float, default=0.15)
    a = ap.parse_args()
    ks, ms = load(a.trace)
    proofs = [m for m in ms if m[2] == "plonk_prove"]
    s, e, _ = proofs[a.proof]
    print("proof %d of %d: %.3f ms" % (a.proof % len(proofs), len(proofs), (e - s) / 1e6))
    for m in ms:
        if s <= m[0] and m[1] <= e and m[2] != "plonk_prove":
            print("%8.3f %8.3f  %s" % ((m[0] - s) / 1e6, (m[1] - s) / 1e6, m[2]))
    end = s
    for k in ks:
        if not s <= k[0] < e:
            continue
        if k[0] > end + a.gap * 1e6:
            print("   --- GPU idle %.3f ms" % ((k[0] - end) / 1e6))
        print("%8.3f %8.3f %7.3f %6s %s" % ((k[0] - s) / 1e6, (k[1] - s) / 1e6, (k[1] - k[0]) / 1e6, k[3], k[2][:60]))
        end = max(end, k[1])


if __name__ == "__main__":
    main()
