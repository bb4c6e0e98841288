#!/bin/bash
# ab_acc.sh plus SQ_INSTS_VALU per setting on the isolated accumulation (acc_probe):
#   gpurun -- bash nzcb-circom_amd/tools/ab_acc_pmc.sh <tag> "<VAR=a>" "<VAR=b>"
set -o pipefail
tag=$1; A=$2; B=$3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cfg in "$A" "$B"; do
  d=gpurun_out/${tag}_pmc_${cfg//[^A-Za-z0-9]/_}
  rm -rf $d
  env $cfg timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $d -o run --output-format csv \
    -- python3 nzcb-circom_amd/tools/acc_probe.py > $d.log 2>&1 || exit $?
done
bash nzcb-circom_amd/tools/ab_acc.sh $tag "$A" "$B"
