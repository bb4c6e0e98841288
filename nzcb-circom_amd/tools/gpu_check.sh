#!/bin/bash
# GPU-box check: the -m gpu suite, then one default bench.py line.
#   gpurun -- bash nzcb-circom_amd/tools/gpu_check.sh <tag> [pytest -k expr]
set -o pipefail
tag=${1:-check}
kexpr=${2:-}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
args=(-u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -p no:cacheprovider)
[ -n "$kexpr" ] && args+=(-k "$kexpr")
timeout -k 10 1000 python3 "${args[@]}" > gpurun_out/${tag}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${tag}_pytest.log
[ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
if [ -z "$kexpr" ]; then
  timeout -k 10 300 python3 bench.py > gpurun_out/${tag}_bench.log 2>&1
  rc=$?
  tail -c 3000 gpurun_out/${tag}_bench.log
  exit $rc
fi
