#!/bin/bash
# Prover GPU tests (fixtures + 2^21 parity) on this build, then a same-box A/B against
# lib/ab/<variant>.so (tools/r4_libab.sh: isolated kernels + bench --steps S alternated).
#   gpurun -- bash nzcb-circom_amd/tools/r4_lat.sh <tag> <variant> <regex> [steps]
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_prover.py tests/test_gpu_fullsize.py tests/test_gpu_wvm.py > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest.log
bash nzcb-circom_amd/tools/r4_libab.sh "$@"
# single-lane timeline of this build (tools/timeline.py)
d=gpurun_out/${tag}_lane1; rm -rf $d
timeout -k 10 240 rocprofv3 --kernel-trace --marker-trace -d $d -o run --output-format csv \
  -- python3 bench.py --lanes 1 --steps 6 --warmup 2 --no-cpu-baseline --no-probe > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
python3 nzcb-circom_amd/tools/timeline.py $d --proof -2 > gpurun_out/${tag}_timeline.txt
python3 nzcb-circom_amd/tools/phase_kernels.py $d > gpurun_out/${tag}_phases.txt 2>&1 || true
head -8 gpurun_out/${tag}_timeline.txt
