#!/bin/bash
# NTT pipeline A/B (NZCB_NTT29 = 0: 8x32 passes, 1: 9x29-resident passes) on one box,
# then the NTT and prover parity tests and one bench line:
#   gpurun -- bash nzcb-circom_amd/tools/ab_ntt.sh <tag>
set -o pipefail
tag=${1:-ntt}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
out=gpurun_out/${tag}_ab.log
: > $out
for v in 0 1 0 1; do
  for L in 21 23; do
    echo -n "NZCB_NTT29=$v " >> $out
    NZCB_NTT29=$v timeout -k 10 120 python3 nzcb-circom_amd/tools/ntt_only.py $L 10 >> $out 2>&1 || exit $?
  done
done
cat $out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prover.py tests/test_gpu_fullsize.py \
  -m gpu -x -q --timeout 600 -p no:cacheprovider -k "ntt or prove or golden or 2p21" \
  > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/${tag}_bench.log 2>&1
rc=$?; tail -c 600 gpurun_out/${tag}_bench.log; exit $rc
