#!/usr/bin/env python3
"""GPU busy time and per-kernel resident time inside the bench's timed window, from a
rocprofv3 --kernel-trace --marker-trace directory (tools/trace_ab.sh). The timed window
is the span of the 40 plonk_prove ranges that run with the most overlap (5 lanes)."""
import collections
import csv
import glob
import os
import sys


def load(d):
    kf = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    mf = glob.glob(os.path.join(d, "**", "*marker_api_trace.csv"), recursive=True)[0]
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", ""))
          for r in csv.DictReader(open(kf))]
    ps = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(mf))
                if r["Function"] == "plonk_prove")
    return ks, ps


def window(ps, k=40):
    best = None
    for i in range(len(ps) - k + 1):
        s, e = ps[i][0], max(p[1] for p in ps[i:i + k])
        if best is None or e - s < best[1] - best[0]:
            best = (s, e)
    return best


def union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def main():
    for d in sys.argv[1:]:
        ks, ps = load(d)
        ws, we = window(ps)
        inside = [(max(s, ws), min(e, we), n) for s, e, n in ks if s < we and e > ws]
        busy = union([(s, e) for s, e, _ in inside])
        per = collections.defaultdict(float)
        for s, e, n in inside:
            per[n] += e - s
        print(f"{d}: window {(we - ws) / 1e6:.2f} ms for 40 proofs, GPU busy {busy / 1e6:.2f} ms "
              f"({100 * busy / (we - ws):.1f} %), kernels {len(inside)}")
        for n, t in sorted(per.items(), key=lambda kv: -kv[1])[:14]:
            print(f"   {n[:64]:64s} {t / 1e6 / 40:8.3f} ms resident per proof")


if __name__ == "__main__":
    main()
