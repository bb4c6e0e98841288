#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV (or rocpd .db): per-kernel time and the GPU busy fraction
(union of kernel intervals) over the trace's last `--window` seconds."""
import argparse
import csv
import collections


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window", type=float, default=0.0, help="only the last N seconds (0 = all)")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--last", nargs=2, metavar=("KERNEL", "COUNT"),
                    help="window from the COUNT-th last launch of a kernel whose name contains KERNEL to its last")
    ap.add_argument("--skip-last", type=int, default=0,
                    help="with --last: end the window before the kernel's last SKIP launches (e.g. a probe)")
    ap.add_argument("--before-last", metavar="NAME", default=None,
                    help="with --last: end the window before the last launch of a kernel whose name contains NAME "
                         "(bench.py's probe starts with k_fixed_base, its random bases)")
    ap.add_argument("--durations", action="store_true",
                    help="with --last: also print the average duration of the KERNEL launches in the window")
    a = ap.parse_args()
    rows = []
    if a.trace.endswith(".db"):  # rocprofv3 >= 7 default output (rocpd SQLite)
        import sqlite3
        con = sqlite3.connect(a.trace)
        rows = [(int(s), int(e), n) for s, e, n in con.execute("select start, end, name from kernels")]
    else:
        with open(a.trace) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    t_end = max(e for _, e, _ in rows)
    if a.last:
        hits = [r for r in rows if a.last[0] in r[2]]
        if a.before_last:
            cut = max(r[0] for r in rows if a.before_last in r[2])
            hits = [r for r in hits if r[1] <= cut]
        if a.skip_last:
            hits = hits[:-a.skip_last]
        hits = hits[-int(a.last[1]):]
        lo, t_end = hits[0][0], hits[-1][1]
        rows = [r for r in rows if lo <= r[0] and r[1] <= t_end]
        if a.durations:
            d = [e - s for s, e, _ in hits]
            print(f"{a.last[0]}: {len(d)} launches, average duration {sum(d) / len(d) / 1e6:.4f} ms, "
                  f"min {min(d) / 1e6:.4f} ms, max {max(d) / 1e6:.4f} ms")
    elif a.window > 0:
        rows = [r for r in rows if r[0] >= t_end - a.window * 1e9]
    t0 = min(s for s, _, _ in rows)
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = t_end - t0
    print(f"span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms ({100 * busy / span:.1f}%), {len(rows)} dispatches")
    agg = collections.defaultdict(lambda: [0, 0])
    for s, e, n in rows:
        k = n.split("(")[0].replace("void ", "")[:70]
        agg[k][0] += e - s
        agg[k][1] += 1
    tot = sum(v[0] for v in agg.values())
    for k, (d, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:a.top]:
        print(f"{k:72s} {c:6d} {d / 1e6:10.2f} ms {d / c / 1e3:9.1f} us {100 * d / tot:5.1f}%")


if __name__ == "__main__":
    main()
