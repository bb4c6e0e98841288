#!/bin/bash
# c = 20 fixed-base window (13 table rows, 2^19 buckets) against c = 17: parity tests under
# NZCB_FB_WINDOW=20, then acc_probe / bench A/B on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NZCB_FB_WINDOW=20 timeout -k 10 900 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prover.py \
  tests/test_gpu_split.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 600 -p no:cacheprovider \
  -k "msm or golden or live or split or 2p21" > gpurun_out/c20_tests.log 2>&1
rc=$?; tail -3 gpurun_out/c20_tests.log; [ $rc -ne 0 ] && exit $rc
bash nzcb-circom_amd/tools/ab_env.sh c20 "NZCB_FB_WINDOW=17" "NZCB_FB_WINDOW=20" bench
