#!/bin/bash
# hardware queues 24 vs 32 at the driver's shape (--steps 20 --warmup 5) and at 300 steps, one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/f; rm -rf $O; mkdir -p $O
for rep in 1 2 3; do for q in 24 32; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe > $O/b.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][-1]);print('q$q steps20', d['value'], d['ms_per_step'], d['single_proof_latency_ms'])"
done; done
for rep in 1 2; do for q in 24 32; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-probe > $O/b.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][-1]);print('q$q steps300', d['value'], d['ms_per_step'], d['single_proof_latency_ms'])"
done; done
GPU_MAX_HW_QUEUES=32 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace -d $O/t -o run --output-format csv \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe > $O/bt.log 2>&1 || exit $?
python3 nzcb-circom_amd/tools/fill_drain.py $O/t 20 20 | tail -3
