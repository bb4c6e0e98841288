#!/bin/bash
# libraries: lib/libnzcb.so built with tools/sessions/r6_ntt_radix8.patch applied to csrc/ntt.hip (NZ_NTT_R8=1),
# lib/ab/libnzcb_r4ntt.so the same source with -DNZ_NTT_R8=0 (the radix-4 plan of the committed kernel)
# radix-8 NTT groups: NTT + kernel tests, isolated NTT times, same-box bench A/B against radix-4
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/d; mkdir -p $O
echo "== pytest $(date +%T)"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prover.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for L in 21 23; do for cfg in r8 r4; do
  Lb=nzcb-circom_amd/lib/libnzcb.so; [ $cfg = r4 ] && Lb=nzcb-circom_amd/lib/ab/libnzcb_r4ntt.so
  echo "$cfg $(NZCB_LIB=$Lb timeout -k 10 120 python3 nzcb-circom_amd/tools/ntt_only.py $L 50)"
done; done
for L in 21; do for cfg in r8 r4 r8 r4; do
  Lb=nzcb-circom_amd/lib/libnzcb.so; [ $cfg = r4 ] && Lb=nzcb-circom_amd/lib/ab/libnzcb_r4ntt.so
  echo "$cfg $(NZCB_LIB=$Lb timeout -k 10 120 python3 nzcb-circom_amd/tools/ntt_only.py $L 200)"
done; done
for cfg in r8 r4 r8 r4; do
  Lb=nzcb-circom_amd/lib/libnzcb.so; [ $cfg = r4 ] && Lb=nzcb-circom_amd/lib/ab/libnzcb_r4ntt.so
  echo "== $cfg $(date +%T)"
  env NZCB_LIB=$Lb timeout -k 10 300 python3 -u bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-probe > $O/ab_$cfg.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads([l for l in open('$O/ab_$cfg.log') if l.startswith('{')][-1]);p=d['phase_ms_single_proof'];print('$cfg', d['value'], d['ms_per_step'], d['single_proof_latency_ms'], [p[k] for k in ('round1','round2','round3','round5')])"
done
