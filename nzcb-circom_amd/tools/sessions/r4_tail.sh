#!/bin/bash
# Round 4 GPU check: the -m gpu suite on the new library, single-lane phase traces of the new
# library and of a variant (lib/ab/<variant>.so), then same-box A/B against the round-3
# library (lib/ab/r3.so): isolated fixed-base MSM phases at 2^21 (tools/acc_probe.py) and
# bench.py alternating r3 / new / variant.
#   gpurun -- bash nzcb-circom_amd/tools/r4_tail.sh <tag> [skip-tests] [steps] [variant]
set -o pipefail
tag=${1:-r4tail}
skip=${2:-}
steps=${3:-120}
variant=${4:-kper4}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}_ab.log
: > $out
if [ -z "$skip" ]; then
  echo "== tests $(date +%T)"
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/${tag}_pytest.log; [ $rc -ne 0 ] && exit $rc
fi
R3=nzcb-circom_amd/lib/ab/r3.so
V=nzcb-circom_amd/lib/ab/${variant}.so
for cfg in "NZCB_FB_WINDOW=20" "NZCB_LIB=$V"; do
  echo "== lane1 [$cfg] $(date +%T)"
  d=gpurun_out/${tag}_lane1
  rm -rf $d
  env $cfg timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace -d $d -o run --output-format csv \
    -- python3 bench.py --lanes 1 --steps 6 --warmup 2 --no-cpu-baseline --no-probe > gpurun_out/${tag}_lane1.log 2>&1 \
    || { tail -20 gpurun_out/${tag}_lane1.log; exit 1; }
  echo "[$cfg]" >> gpurun_out/${tag}_phases.txt
  python3 nzcb-circom_amd/tools/phase_kernels.py $d >> gpurun_out/${tag}_phases.txt || exit 1
  rm -rf $d
done
echo "== acc $(date +%T)"
for rep in 1 2; do
  for cfg in "NZCB_LIB=$R3" "NZCB_FB_WINDOW=17" "NZCB_FB_WINDOW=20"; do
    r=$(env $cfg timeout -k 10 120 python3 nzcb-circom_amd/tools/acc_probe.py --reps 10) || exit 1
    echo "[$cfg] acc: $r" | tee -a $out
  done
done
echo "== bench $(date +%T)"
for rep in 1 2; do
  for cfg in "NZCB_LIB=$R3" "NZCB_FB_WINDOW=20" "NZCB_LIB=$V"; do
    env $cfg timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-probe --steps $steps > gpurun_out/${tag}_bench.log 2>&1 || exit $?
    echo "[$cfg] bench $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/${tag}_bench.log') if l.startswith('{')][-1]);print(d['value'], d['ms_per_step'], d['single_proof_latency_ms'])")" | tee -a $out
  done
done
echo "== node $(date +%T)"
timeout -k 10 600 python3 nzcb-circom_amd/tools/node_bench.py --proofs 120 > gpurun_out/${tag}_node.log 2>&1 || { tail -20 gpurun_out/${tag}_node.log; exit 1; }
tail -1 gpurun_out/${tag}_node.log | tee -a $out
