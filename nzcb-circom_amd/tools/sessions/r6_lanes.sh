#!/bin/bash
# new MSM scalar kinds + real-circuit entry bound, then lanes 4/5/6 same box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/c; mkdir -p $O
echo "== pytest $(date +%T)"
timeout -k 10 800 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_wvm.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in 5 4 6 5 4 6; do
  echo "== lanes $cfg $(date +%T)"
  timeout -k 10 300 python3 -u bench.py --lanes $cfg --steps 300 --warmup 5 --no-cpu-baseline --no-probe > $O/ab_$cfg.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads([l for l in open('$O/ab_$cfg.log') if l.startswith('{')][-1]);print('lanes$cfg', d['value'], d['ms_per_step'], d['single_proof_latency_ms'])"
done
