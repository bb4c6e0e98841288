#!/bin/bash
# NTT A/B on one box over one environment variable (default NZCB_NTT29 = 0: 8x32 passes,
# 1: 9x29-resident passes; e.g. NZCB_NTT_TILE "2048 1024"), alternated, then the NTT and
# prover parity tests under the last value and one bench line:
#   gpurun -- bash nzcb-circom_amd/tools/ab_ntt.sh <tag> [VAR] ["v1 v2"]
set -o pipefail
tag=${1:-ntt}
var=${2:-NZCB_NTT29}
vals=${3:-"0 1"}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
out=gpurun_out/${tag}_ab.log
: > $out
for rep in 1 2; do
  for v in $vals; do
    for L in 21 23; do
      echo -n "$var=$v " >> $out
      env $var=$v timeout -k 10 120 python3 nzcb-circom_amd/tools/ntt_only.py $L 20 >> $out 2>&1 || exit $?
    done
  done
done
cat $out
last=${vals##* }
env $var=$last timeout -k 10 900 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prover.py tests/test_gpu_fullsize.py \
  -m gpu -x -q --timeout 600 -p no:cacheprovider -k "ntt or prove or golden or 2p21" \
  > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_tests.log; [ $rc -ne 0 ] && exit $rc
for v in $vals; do
  env $var=$v timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-probe > gpurun_out/${tag}_bench_$v.log 2>&1
  rc=$?; [ $rc -ne 0 ] && exit $rc
  echo "$var=$v $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/${tag}_bench_$v.log') if l.startswith('{')][-1]);print(d['value'], d['ms_per_step'], d['single_proof_latency_ms'], d['phase_ms_single_proof']['ntt'])")" | tee -a $out
done
