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
WINDOW = 20  # csrc/msm.hip kFbWindow


def pmc_avg(path, counter, last=10):
    """Average of the kernel's last `last` dispatches: bench.py's isolated probe, the same
    launch shape as roofline.avg_launch_ms (the timed region's A, B, C MSMs are smaller)."""
    rows = [(int(r["Dispatch_Id"]), float(r["Counter_Value"])) for r in csv.DictReader(open(path))
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter]
    vals = [v for _, v in sorted(rows)][-last:]
    return len(vals), (sum(vals) / len(vals) if vals else None)


def valu_by_kernel(path):
    """SQ_INSTS_VALU per kernel per proof, dispatches from the first proof on (context
    setup excluded): rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -- bench.py --lanes 1 ..."""
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == "SQ_INSTS_VALU"]
    first = min(int(r["Dispatch_Id"]) for r in rows if "k_wit_to_mont" in r["Kernel_Name"])
    nproofs = sum(1 for r in rows if "k_wit_to_mont" in r["Kernel_Name"])
    agg = {}
    for r in rows:
        if int(r["Dispatch_Id"]) < first:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
        c, v = agg.get(k, (0, 0.0))
        agg[k] = (c + 1, v + float(r["Counter_Value"]))
    tot = sum(v for _, v in agg.values())
    lines = ["# rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -- python3 bench.py --lanes 1 --steps 4 --warmup 1 "
             "--no-cpu-baseline --no-probe",
             f"# dispatches from the first proof on (context setup excluded): {nproofs} proofs (latency/PCIe runs, "
             f"warm-up, timed)",
             f"# {tot / 1e9:.2f} G wave-level VALU instructions, {tot / nproofs / 1e9:.2f} G per proof"]
    for k, (c, v) in sorted(agg.items(), key=lambda x: -x[1][1])[:30]:
        lines.append(f"{k:62s} {c:5d} launches {v / nproofs / 1e9:8.3f} G/proof {100 * v / tot:5.1f}%")
    return "\n".join(lines) + "\n"


def acc_pmc(src, ent):
    """SQ / GRBM counters of the isolated accumulation (tools/acc_probe.py, two passes); ent =
    the probe's bucket entries per launch (bench.py roofline.bucket_entries_per_launch)."""
    vals, lines = {}, ["# rocprofv3 --pmc (two passes) -- python3 nzcb-circom_amd/tools/acc_probe.py",
                       f"# fixed-base MSM alone, 2^21 + 6 points of random scalars, c = {WINDOW}; "
                       "msm_accumulate29_kernel<true>, averages over each pass's launches"]
    for d in ("pmcA", "pmcB"):
        agg = {}
        for f in glob.glob(os.path.join(src, d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if KERNEL in r["Kernel_Name"]:
                    agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        lines.append(f"pass {d[-1]}:")
        for k, v in sorted(agg.items()):
            vals[k] = sum(v) / len(v)
            lines.append(f"  {k:24s} launches {len(v)}  avg {vals[k]:.6g}")
    wc = vals["SQ_WAVE_CYCLES"]
    quad = 1024 * vals["GRBM_GUI_ACTIVE"] / 8 / 4
    lines += ["derived (SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles, MI355X_MICROARCH.md):",
              f"  VALU instructions per bucket entry (lane level) = SQ_INSTS_VALU x 64 / {ent} = "
              f"{vals['SQ_INSTS_VALU'] * 64 / ent:.0f}",
              f"  wave time: issuing {100 * vals['SQ_ACTIVE_INST_ANY'] / wc:.1f} %, issue-stalled (SQ_WAIT_INST_ANY) "
              f"{100 * vals['SQ_WAIT_INST_ANY'] / wc:.1f} %, parked (SQ_WAIT_ANY) {100 * vals['SQ_WAIT_ANY'] / wc:.1f} %",
              f"  GRBM_GUI_ACTIVE / 8 XCDs = {vals['GRBM_GUI_ACTIVE'] / 8 / 1e6:.2f} M cycles per launch",
              f"  {100 * vals['SQ_INSTS_VALU'] / quad:.1f} % of the 1024 SIMDs' quad-cycles issue a VALU instruction "
              f"(v_mad_u64_u32 measures ~5 cycles, profiles/r1_isa_bench.txt: the VALU is saturated)"]
    return "\n".join(lines) + "\n"


def head_commit() -> str:
    try:
        return subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], check=True, capture_output=True,
                              text=True).stdout.strip()
    except (OSError, subprocess.CalledProcessError):
        return "unknown"


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
    summ = subprocess.run([sys.executable, ts, trace, "--last", KERNEL, str(launches), "--before-last", "k_fixed_base",
                           "--durations", "--top", "30"], check=True, capture_output=True, text=True).stdout
    with open(os.path.join(out, f"{a.prefix}_bench_trace_summary.txt"), "w") as f:
        f.write(f"# isolated probe: the last {probe} {KERNEL} launches of the profiled bench.py run "
                f"(bench.py accumulate_probe; roofline.avg_launch_ms = {bench['roofline']['avg_launch_ms']} ms "
                f"from its HIP events)\n" + psumm +
                f"\n# timed window: the {launches} {KERNEL} launches before the probe (its random bases, k_fixed_base, start it) "
                f"(the timed region's proofs x their MSM launches: 7 per proof since round 6, the A, B, C "
                f"commitments being one)\n" + summ)
    nf, fetch_kb = pmc_avg(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    nw, write_kb = pmc_avg(os.path.join(src, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    fetch_raw = fetch_kb * 1024
    traffic = {
        "kernel": "msm_accumulate29_kernel<true> (fixed-base bucket accumulation: LDS-staged indices, paired "
                  "products; 2^21+6-point MSM of random scalars at the default window, c = %d: bench.py's probe, the "
                  "last 10 launches of each pass)" % WINDOW,
        "command": "rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE (separate passes) -- python3 bench.py "
                   "--no-cpu-baseline --steps 8",
        "counters_kb_per_launch": {"FETCH_SIZE": {"launches": nf, "avg_kb_per_launch": round(fetch_kb, 1)},
                                   "WRITE_SIZE": {"launches": nw, "avg_kb_per_launch": round(write_kb, 1)}},
        "correction": "none: random 64-byte gathers are counted at ~1.15x their bytes, not 1/2 "
                      "(profiles/r2_fetch_calibration.txt, tools/gather_calib.hip); FETCH_SIZE + WRITE_SIZE as reported",
        # bench.py puts this into roofline.traffic_source (the run the bytes came from)
        "source": "tools/profile_round.sh, %s profile set, commit %s" % (a.prefix, head_commit()),
        "fetch_bytes_per_launch_raw": int(fetch_raw),
        "bytes_per_launch": int(fetch_raw + write_kb * 1024),
        "note": "gathers are random 64 B affine table points (16 B/lane dwordx4 loads); algorithmic bytes "
                "96 B x 2^21 points = 201 MB; gathered table bytes 64 B x %.1f M entries = %.2f GB"
                % (bench["roofline"]["bucket_entries_per_launch"] / 1e6,
                   bench["roofline"]["bucket_entries_per_launch"] * 64 / 1e9),
    }
    with open(os.path.join(out, "accumulate_traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1)
        f.write("\n")
    pv = os.path.join(src, "pmcv", "run_counter_collection.csv")
    if os.path.exists(pv):
        with open(os.path.join(out, f"{a.prefix}_valu_by_kernel.txt"), "w") as f:
            f.write(valu_by_kernel(pv))
    if os.path.isdir(os.path.join(src, "pmcA")) and os.path.isdir(os.path.join(src, "pmcB")):
        with open(os.path.join(out, f"{a.prefix}_acc_pmc.txt"), "w") as f:
            f.write(acc_pmc(src, bench["roofline"]["bucket_entries_per_launch"]))
    mb = os.path.join(src, "microbench.log")
    if os.path.exists(mb):
        shutil.copy(mb, os.path.join(out, f"{a.prefix}_microbench.txt"))
    lane1 = os.path.join(src, "lane1")
    if os.path.isdir(lane1):   # single-lane kernel breakdown per roctx phase (tools/phase_kernels.py)
        txt = subprocess.run([sys.executable, os.path.join(HERE, "phase_kernels.py"), lane1, "--proofs", "4"],
                             check=True, capture_output=True, text=True).stdout
        with open(os.path.join(out, f"{a.prefix}_single_lane_phases.txt"), "w") as f:
            f.write("# rocprofv3 --kernel-trace --marker-trace -- python3 bench.py --lanes 1 --steps 6 --warmup 2 "
                    "--no-cpu-baseline --no-probe\n" + txt)
    print(psumm + summ)


if __name__ == "__main__":
    main()
