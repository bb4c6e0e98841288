#!/usr/bin/env python3
"""Per-phase kernel breakdown of single-lane proofs.

Input: the CSVs of
  rocprofv3 --kernel-trace --marker-trace --output-format csv -d DIR -o run \
      -- python3 bench.py --lanes 1 ...
With one lane a proof's kernels run inside its roctx phase ranges (csrc/prover.hip
RoctxPhases: "witness", "round1" .. "round5" inside "plonk_prove"). For the last --proofs
plonk_prove ranges this prints each phase's wall time and, per phase, the kernels whose
execution overlaps it: launches, summed duration, and the busy time (union of intervals,
i.e. what runs concurrently is counted once), the top --top kernels by summed duration.
"""
import argparse
import collections
import csv
import glob
import os


def read_csv(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def col(row, *cands):
    for c in cands:
        if c in row:
            return row[c]
    raise KeyError(f"none of {cands} in {list(row)}")


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
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
    ap = argparse.ArgumentParser()
    ap.add_argument("dir", help="rocprofv3 -d output directory (searched recursively for the CSVs)")
    ap.add_argument("--proofs", type=int, default=4)
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    kf = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    mf = glob.glob(os.path.join(a.dir, "**", "*marker_api_trace.csv"), recursive=True)
    if not kf or not mf:
        raise SystemExit(f"kernel or marker trace CSV not found under {a.dir}: {kf} {mf}")
    kernels = [(int(col(r, "Start_Timestamp")), int(col(r, "End_Timestamp")), col(r, "Kernel_Name"))
               for r in read_csv(kf[0])]
    marks = []
    for r in read_csv(mf[0]):
        name = col(r, "Function", "Marker_Message", "Name", "Operation")
        marks.append((int(col(r, "Start_Timestamp")), int(col(r, "End_Timestamp")), name))
    proofs = sorted(m for m in marks if m[2] == "plonk_prove")[-a.proofs:]
    phases = collections.defaultdict(list)     # phase -> [(s, e)] inside the selected proofs
    for s, e, name in marks:
        if name == "plonk_prove" or e <= s:   # instant marks ("mark: ...") are not phases
            continue
        if any(ps <= s and e <= pe for ps, pe, _ in proofs):
            phases[name].append((s, e))
    print(f"# single-lane proofs: {len(proofs)} (last plonk_prove ranges of {os.path.basename(kf[0])})")
    wall = sum(e - s for s, e, _ in proofs) / len(proofs) / 1e6
    print(f"plonk_prove wall {wall:.3f} ms per proof")
    order = sorted(phases, key=lambda n: min(s for s, _ in phases[n]))
    for ph in order:
        iv = phases[ph]
        pw = sum(e - s for s, e in iv) / len(proofs) / 1e6
        hits = collections.defaultdict(list)
        busy = []
        for ks, ke, kn in kernels:
            for s, e in iv:
                if ks < e and ke > s:       # overlaps the phase
                    cs, ce = max(ks, s), min(ke, e)
                    hits[kn.split("(")[0]].append(ce - cs)
                    busy.append((cs, ce))
                    break
        print(f"\n{ph}: wall {pw:.3f} ms per proof, GPU busy {union(busy) / len(proofs) / 1e6:.3f} ms")
        print(f"  {'kernel':64s} {'launches':>8s} {'sum ms':>9s}")
        for kn, d in sorted(hits.items(), key=lambda kv: -sum(kv[1]))[:a.top]:
            print(f"  {kn[:64]:64s} {len(d) / len(proofs):8.1f} {sum(d) / len(proofs) / 1e6:9.3f}")


if __name__ == "__main__":
    main()
