#!/bin/bash
# Round 4 check on one box: the -m gpu suite, one bench.py line (--steps S) and the
# single-lane phase trace (rocprofv3 --kernel-trace --marker-trace, tools/phase_kernels.py).
#   gpurun -- bash nzcb-circom_amd/tools/r4_check.sh <tag> [skip-tests] [steps]
set -o pipefail
tag=${1:-chk}
skip=${2:-}
steps=${3:-200}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -z "$skip" ]; then
  echo "== tests $(date +%T)"
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/${tag}_pytest.log; [ $rc -ne 0 ] && exit $rc
fi
echo "== bench $(date +%T)"
timeout -k 10 400 python3 bench.py --steps $steps > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
grep '^{' gpurun_out/${tag}_bench.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['single_proof_latency_ms'], d['phase_ms_single_proof'])"
echo "== lane1 $(date +%T)"
d=gpurun_out/${tag}_lane1
rm -rf $d
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace -d $d -o run --output-format csv \
  -- python3 bench.py --lanes 1 --steps 6 --warmup 2 --no-cpu-baseline --no-probe > gpurun_out/${tag}_lane1.log 2>&1 \
  || { tail -20 gpurun_out/${tag}_lane1.log; exit 1; }
python3 nzcb-circom_amd/tools/phase_kernels.py $d > gpurun_out/${tag}_phases.txt || exit 1
rm -rf $d
head -3 gpurun_out/${tag}_phases.txt
