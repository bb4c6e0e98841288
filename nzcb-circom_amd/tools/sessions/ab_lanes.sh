#!/bin/bash
# Same-box bench A/B over proof lanes per GPU (bench.py --lanes), alternated twice:
#   gpurun -- bash nzcb-circom_amd/tools/ab_lanes.sh <tag> 5 6 [7 ...]
set -o pipefail
tag=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}_lanes.log
: > $out
for rep in 1 2; do
  for L in "$@"; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --lanes $L --steps 120 > gpurun_out/${tag}_bench.log 2>&1 || exit $?
    echo "[lanes=$L] bench $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/${tag}_bench.log') if l.startswith('{')][-1]);print(d['value'], d['ms_per_step'])")" | tee -a $out
  done
done
