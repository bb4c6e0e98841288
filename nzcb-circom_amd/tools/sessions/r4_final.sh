#!/bin/bash
# End-of-round call: the whole -m gpu suite and one default bench.py line (tools/r4_check.sh
# without its lane trace), then the profiles (tools/profile_r4.sh).
#   gpurun --timeout 1200 -- bash nzcb-circom_amd/tools/r4_final.sh <tag>
set -o pipefail
tag=${1:-final}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "== tests $(date +%T)"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_pytest.log; [ $rc -ne 0 ] && exit $rc
echo "== bench $(date +%T)"
timeout -k 10 300 python3 bench.py > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
grep '^{' gpurun_out/${tag}_bench.log | tail -1 | cut -c1-400
bash nzcb-circom_amd/tools/profile_r4.sh
