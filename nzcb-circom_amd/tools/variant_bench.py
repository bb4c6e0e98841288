"""A/B the library variants in lib/variants/ on the full proof (bench.py) -- one process each."""
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
power = sys.argv[1] if len(sys.argv) > 1 else "21"
for lib in sorted(glob.glob(os.path.join(ROOT, "nzcb-circom_amd", "lib", "variants", "*.so"))):
    env = dict(os.environ, NZCB_LIB=lib)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--power", power, "--steps", "3",
                        "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=300)
    line = [l for l in p.stdout.splitlines() if l.startswith("{")]
    if not line:
        print(os.path.basename(lib), "FAILED", p.stderr[-500:])
        continue
    d = json.loads(line[-1])
    print(os.path.basename(lib), d["value"], d["ms_per_step"], "msm_acc_ms", d["roofline"]["avg_launch_ms"],
          json.dumps(d["phase_ms_last_proof"]), flush=True)
