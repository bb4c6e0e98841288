#!/usr/bin/env python3
"""Fill and drain of the bench's timed window (round 6): from a rocprofv3 --kernel-trace
--marker-trace directory of `bench.py --steps K`, the last K plonk_prove ranges are the timed
proofs. Prints the window, the GPU-busy fraction (union of kernel intervals) and the proofs in
flight per time bin, and how much of the window runs with fewer than all lanes proving.

    python3 tools/fill_drain.py <trace dir> [K] [bin_ms]
"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    bin_ms = float(sys.argv[3]) if len(sys.argv) > 3 else 10.0
    kf = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    mf = glob.glob(os.path.join(d, "**", "*marker_api_trace.csv"), recursive=True)[0]
    ps = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(mf))
                if r["Function"] == "plonk_prove")[-k:]
    t0, t1 = min(p[0] for p in ps), max(p[1] for p in ps)
    ks = sorted((max(int(r["Start_Timestamp"]), t0), min(int(r["End_Timestamp"]), t1))
                for r in csv.DictReader(open(kf))
                if int(r["End_Timestamp"]) > t0 and int(r["Start_Timestamp"]) < t1)
    # union of kernel intervals
    busy, cur_s, cur_e = [], None, None
    for s, e in ks:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy.append((cur_s, cur_e))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy.append((cur_s, cur_e))
    span = (t1 - t0) / 1e6
    tot_busy = sum(e - s for s, e in busy) / 1e6
    print(f"timed proofs {len(ps)}: window {span:.2f} ms, GPU busy {tot_busy:.2f} ms ({100 * tot_busy / span:.1f} %)")
    lanes = max(sum(1 for p in ps if p[0] <= t < p[1]) for t in (q[0] for q in ps))
    nb = int(span / bin_ms) + 1
    under = 0.0
    print(f"{'bin (ms)':>12} {'in flight':>10} {'busy %':>7}")
    for b in range(nb):
        a, z = t0 + int(b * bin_ms * 1e6), min(t1, t0 + int((b + 1) * bin_ms * 1e6))
        if z <= a:
            continue
        mid = (a + z) // 2
        fl = sum(1 for p in ps if p[0] <= mid < p[1])
        bz = sum(max(0, min(e, z) - max(s, a)) for s, e in busy) / (z - a)
        if fl < lanes:
            under += (z - a) / 1e6
        print(f"{b * bin_ms:7.0f}-{(b + 1) * bin_ms:<4.0f} {fl:>10} {100 * bz:>7.1f}")
    print(f"with fewer than {lanes} proofs in flight: {under:.1f} ms of {span:.1f} ({100 * under / span:.1f} %)")
    ends = sorted(p[1] for p in ps)
    print("last proof ends (ms after the first of the last five):",
          [round((e - ends[-5]) / 1e6, 2) for e in ends[-5:]])


if __name__ == "__main__":
    main()
