#!/bin/bash
# Round 4 accumulation A/B: the MSM GPU tests, then tools/acc_probe.py at c = 17, 19, 20 for
# lib/ab/<base>.so and this build, alternated twice, then bench.py alternated twice.
#   gpurun -- bash nzcb-circom_amd/tools/r4_accab.sh <tag> <base> [steps]
set -o pipefail
tag=${1:-accab}
base=${2:-r4a}
steps=${3:-200}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}.txt
: > $out
echo "== tests $(date +%T)"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_pytest.log; [ $rc -ne 0 ] && exit $rc
B=nzcb-circom_amd/lib/ab/${base}.so
echo "== acc $(date +%T)"
for rep in 1 2; do
  for w in 17 19 20; do
    for cfg in "NZCB_LIB=$B" "NZCB_R4=1"; do
      r=$(env $cfg NZCB_FB_WINDOW=$w timeout -k 10 120 python3 nzcb-circom_amd/tools/acc_probe.py --reps 10) || exit 1
      echo "[$cfg c=$w] acc: $r" | tee -a $out
    done
  done
done
line() { python3 -c "import json;d=json.loads([l for l in open('$1') if l.startswith('{')][-1]);print(d['value'], d['ms_per_step'], d['single_proof_latency_ms'])"; }
echo "== bench $(date +%T)"
for rep in 1 2; do
  for cfg in "NZCB_LIB=$B" "NZCB_R4=1"; do
    env $cfg timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-probe --steps $steps > gpurun_out/${tag}_bench.log 2>&1 || exit 1
    echo "[$cfg] bench $(line gpurun_out/${tag}_bench.log)" | tee -a $out
  done
done
