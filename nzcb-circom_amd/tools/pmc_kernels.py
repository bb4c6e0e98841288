#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 output directories: PMC counters (average per launch,
from *counter_collection.csv) and durations (average per launch, from *kernel_trace.csv),
for kernels whose name matches a regular expression.
  python3 tools/pmc_kernels.py <regex> <dir> [<dir> ...]"""
import collections
import csv
import glob
import re
import sys


def main():
    pat = re.compile(sys.argv[1])
    val = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.Counter())
    dur = collections.defaultdict(list)
    for d in sys.argv[2:]:
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "")
                if pat.search(k):
                    val[k][r["Counter_Name"]] += float(r["Counter_Value"])
                    cnt[k][r["Counter_Name"]] += 1
        for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "")
                if pat.search(k):
                    dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for k in sorted(set(val) | set(dur)):
        parts = [f"{c} {val[k][c] / cnt[k][c] / 1e3:9.1f} MB" for c in sorted(val[k])]  # rocprofv3 FETCH/WRITE_SIZE: KB
        if dur[k]:
            parts.append(f"{len(dur[k])} launches avg {sum(dur[k]) / len(dur[k]):.4f} ms")
        print(f"  {k[:48]:48s} " + "  ".join(parts))


if __name__ == "__main__":
    main()
