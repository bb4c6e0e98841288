#!/bin/bash
# Same-box bench A/B over several environment settings, alternated, each run twice
# (BENCH_ARGS: extra bench.py arguments, e.g. "--steps 200" for a longer timed region):
#   gpurun -- bash nzcb-circom_amd/tools/ab_multi.sh <tag> "<VAR=a ...>" "<VAR=b ...>" ...
set -o pipefail
tag=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}_multi.log
: > $out
for rep in 1 2; do
  for cfg in "$@"; do
    env $cfg timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe ${BENCH_ARGS:-} > gpurun_out/${tag}_bench.log 2>&1 || exit $?
    echo "[$cfg] bench $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/${tag}_bench.log') if l.startswith('{')][-1]);print(d['value'], d['ms_per_step'], d['single_proof_latency_ms'])")" | tee -a $out
  done
done
