#!/usr/bin/env python3
"""Node.js boundary throughput: writes the nzcp_live zkey, witness
program and K pass inputs (bench.py's passes), runs js/bench.js (N concurrent
plonk.fullProve calls through the snarkjs-shaped API), checks the first pass's public
signals against the independent nzcp kernel, and prints the Node line.
  python3 tools/node_bench.py [--proofs K] [--concurrency N] [--lanes L] [--dir D] [--reuse]
The GPU work of the preparation runs in a child process (--prep), so the process that
starts node has never initialised the GPU."""
import argparse
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--proofs", type=int, default=120)
    ap.add_argument("--concurrency", type=int, default=10)
    ap.add_argument("--lanes", type=int, default=5)
    ap.add_argument("--dir", default="/tmp/nzcb_node_bench")
    ap.add_argument("--prep", action="store_true")
    ap.add_argument("--reuse", action="store_true", help="keep the files of an earlier run in --dir")
    a = ap.parse_args()
    if not a.prep:
        if a.reuse and os.path.exists(os.path.join(a.dir, "want.json")):
            run_node(a)
            return
        q = subprocess.run([sys.executable, os.path.abspath(__file__), "--prep", "--proofs", str(a.proofs), "--dir",
                            a.dir], timeout=1200)
        if q.returncode:
            sys.exit(q.returncode)
        run_node(a)
        return
    import nzcb
    from nzcb import nzcp, nzcplive
    import bench
    os.makedirs(a.dir, exist_ok=True)
    r1cs, prog, _ = nzcplive.build()
    zp, zl = nzcplive.setup_raw(r1cs)
    try:
        with open(os.path.join(a.dir, "live.zkey"), "wb") as f:
            f.write((ctypes.c_uint8 * zl).from_address(zp))
    finally:
        nzcb.free_ptr(zp)
    with open(os.path.join(a.dir, "live.nzwp"), "wb") as f:
        f.write(prog)
    tbs = nzcp.pass_tbs(live=True)
    inputs = [nzcp.circuit_input(tbs, bench.pass_data(i)) for i in range(a.proofs)]
    with open(os.path.join(a.dir, "inputs.json"), "w") as f:
        json.dump(inputs, f)
    rec = nzcb.nzcp_witness(bench.pass_inputs([0]), 1, nzcb.NZCP_LIVE, 0)[0]
    with open(os.path.join(a.dir, "want.json"), "w") as f:
        json.dump([str(v) for v in rec["out"]], f)


def run_node(a):
    with open(os.path.join(a.dir, "want.json")) as f:
        want = json.load(f)
    p = subprocess.run(["node", os.path.join(PKG, "js", "bench.js"), os.path.join(a.dir, "live.zkey"),
                        os.path.join(a.dir, "live.nzwp"), os.path.join(a.dir, "inputs.json"), str(a.concurrency),
                        str(a.lanes)], capture_output=True, text=True, timeout=1200)
    sys.stderr.write(p.stderr)
    if p.returncode:
        print(p.stdout)
        sys.exit(p.returncode)
    line = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
    line["public_signals_match_nzcp_kernel"] = line.pop("publicSignals0") == want
    print(json.dumps(line))
    if not line["public_signals_match_nzcp_kernel"]:
        sys.exit(1)


if __name__ == "__main__":
    main()
