#!/bin/bash
# Round 4: the prover GPU tests (coalesced evaluations), the SERIAL trace of round 4's
# kernels, then the stream-priority bench A/B (tools/r4_envab.sh).
set -o pipefail
tag=${1:-evp}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "== tests $(date +%T)"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_prover.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 400 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_pytest.log; [ $rc -ne 0 ] && exit $rc
d=gpurun_out/${tag}_serial; rm -rf $d
NZCB_SERIAL=1 timeout -k 10 240 rocprofv3 --kernel-trace -d $d -o run --output-format csv \
  -- python3 bench.py --lanes 1 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
python3 nzcb-circom_amd/tools/pmc_kernels.py 'k_eval|k_pol_r|k_perm|k_lin|k_tile|k_pow' $d > gpurun_out/${tag}_serial.txt || exit 1
rm -rf $d
cat gpurun_out/${tag}_serial.txt
bash nzcb-circom_amd/tools/r4_envab.sh ${tag}_prio 200 "NZCB_R4=1" "NZCB_STREAM_PRIO=1" "NZCB_STREAM_PRIO=2"
