#!/bin/bash
# One profiling call for profiles/ (on the GPU box, from the repo root), then
# `python3 nzcb-circom_amd/tools/collect_profiles.py --prefix rN` here:
#   prof/       rocprofv3 --kernel-trace --stats of the default bench.py run
#   pmc_fetch/  FETCH_SIZE, pmc_write/ WRITE_SIZE (separate passes, bench.py --steps 8)
#   pmcv/       SQ_INSTS_VALU SQ_WAVES by kernel, one lane (where the VALU goes per proof)
#   pmcA/ pmcB/ the isolated accumulation's SQ and GRBM counters (tools/acc_probe.py)
#   lane1/      kernel + roctx marker trace of single-lane proofs (tools/phase_kernels.py)
#   microbench.log  MSM and NTT 2^18..2^24 (configs[1])
# Each step has its own time limit; the first failure ends the call.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmcv gpurun_out/pmcA gpurun_out/pmcB \
  gpurun_out/lane1
step() { echo "== $1 $(date +%T)"; }
step trace
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv \
  -- python3 bench.py > gpurun_out/prof_bench.log 2>&1 || exit $?
step fetch
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv \
  -- python3 bench.py --no-cpu-baseline --steps 8 > gpurun_out/pmc_fetch.log 2>&1 || exit $?
step write
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv \
  -- python3 bench.py --no-cpu-baseline --steps 8 > gpurun_out/pmc_write.log 2>&1 || exit $?
step valu
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d gpurun_out/pmcv -o run --output-format csv \
  -- python3 bench.py --lanes 1 --steps 4 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/pmcv.log 2>&1 || exit $?
step accA
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_WAVES SQ_WAVE_CYCLES -d gpurun_out/pmcA -o run --output-format csv \
  -- python3 nzcb-circom_amd/tools/acc_probe.py > gpurun_out/pmcA.log 2>&1 || exit $?
step accB
timeout -s KILL 120 rocprofv3 --pmc GRBM_COUNT GRBM_GUI_ACTIVE SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
  SQ_INST_CYCLES_VMEM_RD -d gpurun_out/pmcB -o run --output-format csv \
  -- python3 nzcb-circom_amd/tools/acc_probe.py > gpurun_out/pmcB.log 2>&1 || exit $?
step lane1
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace -d gpurun_out/lane1 -o run --output-format csv \
  -- python3 bench.py --lanes 1 --steps 6 --warmup 2 --no-cpu-baseline --no-probe > gpurun_out/lane1.log 2>&1 \
  || exit $?
step microbench
timeout -k 10 300 python3 -u nzcb-circom_amd/tools/microbench.py > gpurun_out/microbench.log 2>&1 || exit $?
step done
echo profile-ok
