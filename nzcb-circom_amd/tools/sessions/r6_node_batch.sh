#!/bin/bash
# Node boundary throughput and the configs[3] 512-proof batch at the final round-6 code, one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/i; rm -rf $O; mkdir -p $O
echo "== bench $(date +%T)"
timeout -k 10 300 python3 -u bench.py --steps 120 --warmup 5 --no-cpu-baseline --no-probe > $O/b120.log 2>&1 || exit $?
python3 -c "import json;d=json.loads([l for l in open('$O/b120.log') if l.startswith('{')][-1]);print('bench.py steps120', d['value'], d['ms_per_step'])"
echo "== node $(date +%T)"
for c in 10 16; do
  timeout -k 10 400 python3 -u nzcb-circom_amd/tools/node_bench.py --proofs 120 --concurrency $c $([ $c = 16 ] && echo --reuse) > $O/node$c.log 2>&1 || exit $?
  tail -2 $O/node$c.log
done
echo "== batch512 $(date +%T)"
timeout -k 10 400 python3 -u bench.py --batch 512 --no-cpu-baseline --no-probe > $O/b512.log 2>&1 || exit $?
grep '^{"metric"' $O/b512.log | tail -1 | cut -c1-300
