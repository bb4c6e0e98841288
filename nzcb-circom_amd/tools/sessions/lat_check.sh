#!/bin/bash
# GPU-box check of an MSM change: a -m gpu subset, the single-lane phase trace
# (tools/phase_kernels.py reads gpurun_out/<tag>_lane1), then one default bench.py line.
#   gpurun -- bash nzcb-circom_amd/tools/lat_check.sh <tag> [pytest -k expr]
set -o pipefail
tag=${1:-lat}
kexpr=${2:-"msm or prove or lagrange or split"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -rf gpurun_out/${tag}_lane1
echo "== tests $(date +%T)"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "$kexpr" > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest.log
echo "== lane1 $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace -d gpurun_out/${tag}_lane1 -o run --output-format csv \
  -- python3 bench.py --lanes 1 --steps 6 --warmup 2 --no-cpu-baseline --no-probe > gpurun_out/${tag}_lane1.log 2>&1 \
  || { tail -20 gpurun_out/${tag}_lane1.log; exit 1; }
python3 nzcb-circom_amd/tools/phase_kernels.py gpurun_out/${tag}_lane1 > gpurun_out/${tag}_phases.txt || exit 1
rm -rf gpurun_out/${tag}_lane1
echo "== bench $(date +%T)"
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
tail -c 1500 gpurun_out/${tag}_bench.log
echo lat-check-ok
