#!/bin/bash
# the driver's bench shape (--steps 20 --warmup 5): kernel + marker trace for the timed window's fill and drain
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/e; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace -d $O/t -o run --output-format csv \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe > $O/b.log 2>&1 || exit $?
grep '^{"metric"' $O/b.log | cut -c1-200
for s in 20 300; do
  timeout -k 10 300 python3 bench.py --steps $s --warmup 5 --no-cpu-baseline --no-probe > $O/b$s.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads([l for l in open('$O/b$s.log') if l.startswith('{')][-1]);print('steps$s', d['value'], d['ms_per_step'])"
done
