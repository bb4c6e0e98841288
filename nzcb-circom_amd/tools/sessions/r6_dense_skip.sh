#!/bin/bash
# dense tables skip the min-form: MSM + prover GPU tests, then same-box A/B (new / flipall / r5)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/b; mkdir -p $O
echo "== pytest $(date +%T)"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prover.py tests/test_gpu_wvm.py tests/test_gpu_split.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in new flipall r5 new flipall r5; do
  L=nzcb-circom_amd/lib/libnzcb.so; [ $cfg = r5 ] && L=nzcb-circom_amd/lib/ab/libnzcb_r5.so; [ $cfg = flipall ] && L=nzcb-circom_amd/lib/ab/libnzcb_flipall.so
  echo "== $cfg $(date +%T)"
  env NZCB_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-probe > $O/ab_$cfg.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads([l for l in open('$O/ab_$cfg.log') if l.startswith('{')][-1]);p=d['phase_ms_single_proof'];print('$cfg', d['value'], d['ms_per_step'], d['single_proof_latency_ms'], [p[k] for k in ('round1','round2','round3','round5')])"
done
