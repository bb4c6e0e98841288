#!/bin/bash
# Same-box bench.py A/B over environment settings, alternated twice:
#   gpurun -- bash nzcb-circom_amd/tools/r4_envab.sh <tag> <steps> "<VAR=a ...>" ["<VAR=b ...>" ...]
set -o pipefail
tag=$1; shift
steps=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}.txt
: > $out
line() { python3 -c "import json;d=json.loads([l for l in open('$1') if l.startswith('{')][-1]);print(d['value'], d['ms_per_step'], d['single_proof_latency_ms'])"; }
for rep in 1 2; do
  for cfg in "$@"; do
    env $cfg timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-probe --steps $steps > gpurun_out/${tag}_bench.log 2>&1 \
      || { tail -5 gpurun_out/${tag}_bench.log; exit 1; }
    echo "[$cfg] bench $(line gpurun_out/${tag}_bench.log)" | tee -a $out
  done
done
