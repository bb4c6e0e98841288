#!/usr/bin/env python3
"""Copy a profiling call's outputs (gpurun_out/) into profiles/ under a round prefix:

  <prefix>_bench_kernel_stats.csv   rocprofv3 --kernel-trace --stats of the default bench.py run
  <prefix>_bench_trace_summary.txt  tools/trace_summary.py over the timed window (last K accumulations)
  <prefix>_bench_line.txt           that run's bench.py JSON line
  accumulate_traffic.json           FETCH_SIZE / WRITE_SIZE passes of the same kernel (HBM bytes per launch)
  <prefix>_microbench.txt           tools/microbench.py lines (configs[1])

    python3 tools/collect_profiles.py --prefix r1 --src gpurun_out
"""
import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
KERNEL = "msm_accumulate29"


def pmc_avg(path, counter, last=10):
    """Average of the kernel's last `last` dispatches: bench.py's isolated probe, the same
    launch shape as roofline.avg_launch_ms (the timed region's A, B, C MSMs are smaller)."""
    rows = [(int(r["Dispatch_Id"]), float(r["Counter_Value"])) for r in csv.DictReader(open(path))
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter]
    vals = [v for _, v in sorted(rows)][-last:]
    return len(vals), (sum(vals) / len(vals) if vals else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prefix", default="r1")
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--prof", default="prof")
    a = ap.parse_args()
    out = os.path.join(ROOT, "profiles")
    src = a.src
    prof = os.path.join(src, a.prof)
    shutil.copy(os.path.join(prof, "run_kernel_stats.csv"), os.path.join(out, f"{a.prefix}_bench_kernel_stats.csv"))
    line = [l for l in open(os.path.join(src, f"{a.prof}_bench.log")) if l.startswith('{"metric"')][-1]
    bench = json.loads(line)
    with open(os.path.join(out, f"{a.prefix}_bench_line.txt"), "w") as f:
        f.write("# rocprofv3 --kernel-trace --stats -- python3 bench.py   (defaults)\n" + line)
    launches = bench["roofline"]["launches_timed"]
    probe = 10   # bench.py accumulate_probe: 2 + 1 warm-up and 10 timed launches, the last of the run
    ts = os.path.join(HERE, "trace_summary.py")
    trace = os.path.join(prof, "run_kernel_trace.csv")
    psumm = subprocess.run([sys.executable, ts, trace, "--last", KERNEL, str(probe), "--durations", "--top", "12"],
                           check=True, capture_output=True, text=True).stdout
    summ = subprocess.run([sys.executable, ts, trace, "--last", KERNEL, str(launches), "--skip-last", str(probe + 3),
                           "--durations", "--top", "30"], check=True, capture_output=True, text=True).stdout
    with open(os.path.join(out, f"{a.prefix}_bench_trace_summary.txt"), "w") as f:
        f.write(f"# isolated probe: the last {probe} {KERNEL} launches of the profiled bench.py run "
                f"(bench.py accumulate_probe; roofline.avg_launch_ms = {bench['roofline']['avg_launch_ms']} ms "
                f"from its HIP events)\n" + psumm +
                f"\n# timed window: the {launches} {KERNEL} launches before the probe (40 proofs x 9 MSMs)\n" + summ)
    nf, fetch_kb = pmc_avg(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    nw, write_kb = pmc_avg(os.path.join(src, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    fetch_raw = fetch_kb * 1024
    traffic = {
        "kernel": "msm_accumulate29_kernel<4> (fixed-base bucket accumulation, 2^21+6-point MSM of random scalars, "
                  "c=17: bench.py's probe, the last 10 launches of each pass)",
        "command": "rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE (separate passes) -- python3 bench.py "
                   "--no-cpu-baseline --steps 8",
        "counters_kb_per_launch": {"FETCH_SIZE": {"launches": nf, "avg_kb_per_launch": round(fetch_kb, 1)},
                                   "WRITE_SIZE": {"launches": nw, "avg_kb_per_launch": round(write_kb, 1)}},
        "correction": "none: random 64-byte gathers are counted at ~1.15x their bytes, not 1/2 "
                      "(profiles/r2_fetch_calibration.txt, tools/gather_calib.hip); FETCH_SIZE + WRITE_SIZE as reported",
        "fetch_bytes_per_launch_raw": int(fetch_raw),
        "bytes_per_launch": int(fetch_raw + write_kb * 1024),
        "note": "gathers are random 64 B affine table points (16 B/lane dwordx4 loads); algorithmic bytes "
                "96 B x 2^21 points = 201 MB; gathered table bytes 64 B x 31.5 M entries = 2.0 GB",
    }
    with open(os.path.join(out, "accumulate_traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1)
        f.write("\n")
    mb = os.path.join(src, "microbench.log")
    if os.path.exists(mb):
        shutil.copy(mb, os.path.join(out, f"{a.prefix}_microbench.txt"))
    print(psumm + summ)


if __name__ == "__main__":
    main()
