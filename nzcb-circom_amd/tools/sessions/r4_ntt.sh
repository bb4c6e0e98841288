#!/bin/bash
# Round 4 NTT plan A/B: the NTT and MSM GPU tests, the microbenchmarks under the default plan
# (2048-element tiles, two passes for 17 <= log n <= 22) and under NZCB_NTT_TILE=1024 (round
# 3's plan), then bench.py alternating the two.
#   gpurun -- bash nzcb-circom_amd/tools/r4_ntt.sh <tag> [steps]
set -o pipefail
tag=${1:-ntt}
steps=${2:-200}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}.txt
: > $out
echo "== tests $(date +%T)"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prover.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_pytest.log; [ $rc -ne 0 ] && exit $rc
echo "== micro $(date +%T)"
for cfg in "NZCB_R4=1" "NZCB_NTT_TILE=1024"; do
  env $cfg timeout -k 10 600 python3 nzcb-circom_amd/tools/microbench.py > gpurun_out/${tag}_micro.log 2>&1 || { tail -5 gpurun_out/${tag}_micro.log; exit 1; }
  echo "[$cfg] microbench" >> $out
  cat gpurun_out/${tag}_micro.log >> $out
done
line() { python3 -c "import json;d=json.loads([l for l in open('$1') if l.startswith('{')][-1]);print(d['value'], d['ms_per_step'], d['single_proof_latency_ms'], d['phase_ms_single_proof'])"; }
echo "== bench $(date +%T)"
for rep in 1 2; do
  for cfg in "NZCB_R4=1" "NZCB_NTT_TILE=1024"; do
    env $cfg timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-probe --steps $steps > gpurun_out/${tag}_bench.log 2>&1 || exit 1
    echo "[$cfg] bench $(line gpurun_out/${tag}_bench.log)" | tee -a $out
  done
done
