#!/bin/bash
# Same-box A/B of environment switches on the isolated kernels and the bench:
#   gpurun -- bash nzcb-circom_amd/tools/ab_env.sh <tag> "<VAR=a VAR2=b>" "<VAR=c ...>" [bench]
# runs tools/acc_probe.py (fixed-base MSM at 2^21) and tools/ntt_only.py (2^23) twice per
# setting, alternating, then (with "bench") bench.py --no-cpu-baseline --no-probe per setting.
set -o pipefail
tag=$1; A=$2; B=$3; bench=${4:-}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
out=gpurun_out/${tag}_ab.log
: > $out
for rep in 1 2; do
  for cfg in "$A" "$B"; do
    echo "[$cfg] acc: $(env $cfg timeout -k 10 120 python3 nzcb-circom_amd/tools/acc_probe.py --reps 10)" >> $out || exit 1
    echo "[$cfg] $(env $cfg timeout -k 10 120 python3 nzcb-circom_amd/tools/ntt_only.py 23 10)" >> $out || exit 1
  done
done
cat $out
if [ -n "$bench" ]; then
  for cfg in "$A" "$B" "$A" "$B"; do
    env $cfg timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe > gpurun_out/${tag}_bench.log 2>&1 || exit $?
    echo "[$cfg] bench $(python3 -c "import json,sys;d=json.loads([l for l in open('gpurun_out/${tag}_bench.log') if l.startswith('{')][-1]);print(d['value'], d['ms_per_step'])")" | tee -a $out
  done
fi
