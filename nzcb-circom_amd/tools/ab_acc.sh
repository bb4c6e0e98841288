#!/bin/bash
# A/B of the accumulation kernel variants on one box (isolated fixed-base MSM, 2^21 + 6
# points), then the MSM parity tests and one default bench line:
#   gpurun -- bash nzcb-circom_amd/tools/ab_acc.sh <tag>
set -o pipefail
tag=${1:-ab}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
out=gpurun_out/${tag}_ab.log
: > $out
for v in 0 1 0 1; do
  echo "NZCB_ACC_LDS=$v" >> $out
  NZCB_ACC_LDS=$v timeout -k 10 120 python3 nzcb-circom_amd/tools/acc_probe.py --reps 10 >> $out 2>&1 || exit $?
done
cat $out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 -k "msm" \
  -p no:cacheprovider > gpurun_out/${tag}_msm_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_msm_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/${tag}_bench.log 2>&1
rc=$?; tail -c 1500 gpurun_out/${tag}_bench.log; exit $rc
