cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/prof_pair
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pair/kt -o kt --output-format csv -- python3 nzcb-circom_amd/tools/pair_sweep.py --rounds 1 --reps 2 > gpurun_out/prof_pair/kt.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS -d gpurun_out/prof_pair/pmc1 -o pmc1 --output-format csv -- python3 nzcb-circom_amd/tools/pair_sweep.py --rounds 1 --reps 1 > gpurun_out/prof_pair/pmc1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_pair/pmc2 -o pmc2 --output-format csv -- python3 nzcb-circom_amd/tools/pair_sweep.py --rounds 1 --reps 1 > gpurun_out/prof_pair/pmc2.log 2>&1
echo rc=$?
find gpurun_out/prof_pair -name "*.csv" | head
