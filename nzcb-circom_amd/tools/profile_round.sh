#!/bin/bash
# One profiling call for profiles/ (run on the GPU box from the repo root, then
# `python3 nzcb-circom_amd/tools/collect_profiles.py --prefix rN` here):
#   kernel trace + stats of the default bench.py run, FETCH_SIZE and WRITE_SIZE in
#   separate --pmc passes, and the MSM/NTT microbench (configs[1]).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv \
  -- python3 bench.py > gpurun_out/prof_bench.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv \
  -- python3 bench.py --no-cpu-baseline --steps 8 > gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv \
  -- python3 bench.py --no-cpu-baseline --steps 8 > gpurun_out/pmc_write.log 2>&1
timeout -k 10 300 python3 -u nzcb-circom_amd/tools/microbench.py > gpurun_out/microbench.log 2>&1
echo profile-ok
