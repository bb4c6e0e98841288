#!/bin/bash
# (1) bench.py --msm-split as 2 ranks over gloo on one GPU (both ranks on cuda:0; the
#     launcher starts the ranks as fresh processes before any GPU call), and
# (2) SQ counters of the 2^23 NTT passes (tools/ntt_only.py), one --pmc pass each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -rf gpurun_out/ntt_pmcA gpurun_out/ntt_pmcB
NZCB_DIST_BACKEND=gloo NZCB_BENCH_DEVICE=0 timeout -k 10 600 python3 -m torch.distributed.run --nnodes 1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --msm-split --steps 6 \
  --warmup 2 --no-cpu-baseline --no-probe > gpurun_out/split_gloo2.log 2>&1 || exit $?
grep '^{"metric"' gpurun_out/split_gloo2.log | tail -1 | cut -c1-600
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY \
  SQ_ACTIVE_INST_VALU SQ_INSTS_LDS -d gpurun_out/ntt_pmcA -o run --output-format csv \
  -- python3 nzcb-circom_amd/tools/ntt_only.py 23 5 > gpurun_out/ntt_pmcA.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS \
  SQ_INST_CYCLES_VMEM_RD -d gpurun_out/ntt_pmcB -o run --output-format csv \
  -- python3 nzcb-circom_amd/tools/ntt_only.py 23 5 > gpurun_out/ntt_pmcB.log 2>&1 || exit $?
echo split-ntt-ok
