#!/bin/bash
# Kernel traces of the default 5-lane bench under two libraries/settings (same box), for
# tools/trace_gaps.py: gpurun -- bash nzcb-circom_amd/tools/trace_ab.sh <tag> "<env A>" "<env B>"
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for cfg in "$@"; do
  d=gpurun_out/${tag}_tr$i
  rm -rf $d
  env $cfg timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace -d $d -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-probe > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  echo "[$cfg] $(grep -o '"value": [0-9.]*' $d.log)"
  i=$((i + 1))
done
