#!/usr/bin/env python3
"""Time forward NTTs of 2^L on one device (profiling helper: rocprofv3 -- python3 ntt_only.py L reps)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nzcb  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 23
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
e = nzcb.Engine(0, max_log_ntt=L, max_msm_points=16)
a, b = nzcb.dev_alloc((1 << L) * 32), nzcb.dev_alloc((1 << L) * 32)
e.random_fr(a, 1 << L, 1)
print(f"ntt 2^{L}: {e.time_ntt(a, b, L, False, reps):.4f} ms")
