#!/bin/bash
# sign-flip check: MSM + prover GPU tests, stats census, then same-box A/B (new / sparse / r5)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/a; mkdir -p $O
echo "== pytest $(date +%T)"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prover.py tests/test_gpu_wvm.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== stats $(date +%T)"
NZCB_LIB=nzcb-circom_amd/lib/ab/libnzcb_stats.so timeout -k 10 300 python3 -u bench.py --lanes 1 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > $O/stats.log 2>&1 || exit $?
grep -E "MSMSTATS n=2097154|MSMSCALARS" $O/stats.log | sort | uniq -c | sort -rn | head -8
for cfg in new r5 sparse new r5 sparse; do
  L=nzcb-circom_amd/lib/libnzcb.so; E=""; [ $cfg = r5 ] && L=nzcb-circom_amd/lib/ab/libnzcb_r5.so; [ $cfg = sparse ] && E="NZCB_SPARSE=1"
  echo "== $cfg $(date +%T)"
  env NZCB_LIB=$L $E timeout -k 10 300 python3 -u bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-probe > $O/ab_$cfg.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads([l for l in open('$O/ab_$cfg.log') if l.startswith('{')][-1]);p=d['phase_ms_single_proof'];print('$cfg', d['value'], d['ms_per_step'], d['single_proof_latency_ms'], [p[k] for k in ('round1','round2','round3','round5')])"
done
