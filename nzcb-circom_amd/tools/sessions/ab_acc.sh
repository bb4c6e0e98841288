#!/bin/bash
# Accumulation-kernel A/B: the fixed-base MSM and full-size parity tests under the
# candidate setting B, then tools/ab_env.sh (acc_probe + NTT twice each, alternating,
# then the bench per setting) on the same box:
#   gpurun -- bash nzcb-circom_amd/tools/ab_acc.sh <tag> "<VAR=a>" "<VAR=b>"
set -o pipefail
tag=$1; A=$2; B=$3
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
env $B timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_prover.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "msm or golden or 2p21 or 2p24" > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_tests.log; [ $rc -ne 0 ] && exit $rc
bash nzcb-circom_amd/tools/ab_env.sh $tag "$A" "$B" bench
