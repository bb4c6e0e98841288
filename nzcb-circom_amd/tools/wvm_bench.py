#!/usr/bin/env python3
"""Time the GPU witness VM on the nzcp_live program (batches of live-shaped passes)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "nzcb-circom_amd")]
import bench  # noqa: E402
import nzcb  # noqa: E402
from nzcb import nzcplive  # noqa: E402

r1cs, prog, _ = nzcplive.build()
wp = nzcb.WitnessProgram(prog)
print(f"program: {wp.n_wires} wires, {wp.n_levels} levels, {len(prog)} bytes", flush=True)
for count in (1, 8, 40, 256):
    inputs = bench.pass_inputs(range(count))
    din = nzcb.dev_alloc(len(inputs))
    dw = nzcb.dev_alloc(count * wp.n_wires * 32)
    nzcb.h2d(din, inputs)
    wp.run_dev(din, count, dw, wp.n_wires * 32)
    t = time.perf_counter()
    reps = 5
    for _ in range(reps):
        st = wp.run_dev(din, count, dw, wp.n_wires * 32)
    ms = (time.perf_counter() - t) / reps * 1e3
    assert not any(st)
    print(f"passes {count:4d}: {ms:8.3f} ms per batch, {ms / count:7.3f} ms per pass", flush=True)
    nzcb.dev_free(din)
    nzcb.dev_free(dw)
wp.close()
