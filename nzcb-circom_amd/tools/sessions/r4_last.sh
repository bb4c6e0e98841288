#!/bin/bash
# Last call of the round: the prover GPU tests and one default bench line on the in-tree build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_prover.py tests/test_gpu_fullsize.py > gpurun_out/last_pytest.log 2>&1 || { tail -30 gpurun_out/last_pytest.log; exit 1; }
tail -1 gpurun_out/last_pytest.log
timeout -k 10 300 python3 bench.py > gpurun_out/last_bench.log 2>&1 || { tail -20 gpurun_out/last_bench.log; exit 1; }
grep '^{' gpurun_out/last_bench.log | tail -1 | cut -c1-300
