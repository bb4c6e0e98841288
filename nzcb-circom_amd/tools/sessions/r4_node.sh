#!/bin/bash
# Round 4: the Node.js boundary against bench.py on one box, the fixed-batch bench line
# (configs[3]: --batch 512) and the microbenchmarks.
#   gpurun -- bash nzcb-circom_amd/tools/r4_node.sh <tag> [proofs]
set -o pipefail
tag=${1:-node}
proofs=${2:-300}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}.log
: > $out
echo "== node tests $(date +%T)"
timeout -k 10 400 python3 -u -m pytest tests/test_node.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_pytest.log; [ $rc -ne 0 ] && exit $rc
echo "== bench $(date +%T)"
timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-probe --steps 200 > gpurun_out/${tag}_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/${tag}_bench.log | tail -1 >> $out
echo "== node $(date +%T)"
reuse=
for c in 10 16; do
  timeout -k 10 600 python3 nzcb-circom_amd/tools/node_bench.py --proofs $proofs --concurrency $c $reuse > gpurun_out/${tag}_node$c.log 2>&1 \
    || { tail -20 gpurun_out/${tag}_node$c.log; exit 1; }
  tail -1 gpurun_out/${tag}_node$c.log | tee -a $out
  reuse=--reuse
done
echo "== batch 512 $(date +%T)"
timeout -k 10 600 python3 bench.py --gpus 1 --batch 512 > gpurun_out/${tag}_b512.log 2>&1 || exit $?
grep '^{' gpurun_out/${tag}_b512.log | tail -1 >> $out
echo "== microbench $(date +%T)"
timeout -k 10 600 python3 nzcb-circom_amd/tools/microbench.py > gpurun_out/${tag}_micro.log 2>&1 || { tail -20 gpurun_out/${tag}_micro.log; exit 1; }
echo done >> $out
