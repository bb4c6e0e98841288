#!/bin/bash
# GPU box: the whole -m gpu suite, one default bench line, then SQ_INSTS_VALU per kernel
# of single-lane proofs (tools/collect_profiles.py reads gpurun_out/pmcv):
#   gpurun -- bash nzcb-circom_amd/tools/valu_proof.sh <tag>
set -o pipefail
tag=${1:-vp}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "== tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest.log
echo "== bench $(date +%T)"
timeout -k 10 300 python3 bench.py > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
echo "== valu $(date +%T)"
rm -rf gpurun_out/pmcv
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d gpurun_out/pmcv -o run --output-format csv \
  -- python3 bench.py --lanes 1 --steps 4 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/pmcv.log 2>&1 || exit 1
tail -c 1200 gpurun_out/${tag}_bench.log
echo valu-proof-ok
