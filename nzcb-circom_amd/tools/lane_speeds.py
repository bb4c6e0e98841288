#!/usr/bin/env python3
"""Per-lane proof durations of the last K proofs of a rocprofv3 --marker-trace directory
(the "lane k" mark each proof records before its plonk_prove range, on the same thread)."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
mf = glob.glob(os.path.join(d, "**", "*marker_api_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(mf)), key=lambda r: int(r["Start_Timestamp"]))
last_mark = {}
proofs = []
for r in rows:
    if r["Function"].startswith("lane "):
        last_mark[r["Thread_Id"]] = int(r["Function"].split()[1])
    elif r["Function"] == "plonk_prove":
        proofs.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), last_mark.get(r["Thread_Id"], -1)))
proofs = proofs[-k:]
t0 = min(p[0] for p in proofs)
by = collections.defaultdict(list)
for s, e, lane in proofs:
    by[lane].append((s - t0, e - t0))
for lane in sorted(by):
    v = by[lane]
    print(f"lane {lane}: {len(v)} proofs, ms {[round((e - s) / 1e6, 1) for s, e in v]}, last ends {v[-1][1] / 1e6:.1f}")
print(f"window {max(p[1] for p in proofs) / 1e6 - t0 / 1e6:.1f} ms")
