#!/bin/bash
# Prover-level A/B: the whole -m gpu suite under the candidate setting B, then the bench
# (--no-cpu-baseline --no-probe) alternating A, B, A, B on the same box:
#   gpurun -- bash nzcb-circom_amd/tools/ab_prove.sh <tag> "<VAR=a>" "<VAR=b>" [bench args]
set -o pipefail
tag=$1; A=$2; B=$3; shift 3
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
env $B timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_tests.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/${tag}_ab.log
: > $out
for cfg in "$A" "$B" "$A" "$B"; do
  env $cfg timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe "$@" > gpurun_out/${tag}_bench.log 2>&1 || exit $?
  echo "[$cfg] bench $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/${tag}_bench.log') if l.startswith('{')][-1]);print(d['value'], d['ms_per_step'], d['single_proof_latency_ms'], d['phase_ms_single_proof'])")" | tee -a $out
done
