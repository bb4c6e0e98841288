#!/bin/bash
# round 6: sparse accumulation with LDS-staged indices; parity, then same-box A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; O=gpurun_out/r6i; rm -rf $O; mkdir -p $O
echo "== ab $(date +%T)"
run() {  # name lib env...
  local name=$1 lib=$2; shift 2
  env NZCB_LIB=$lib "$@" timeout -k 10 300 python3 -u bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-probe > $O/ab_$name.log 2>&1 || return $?
  python3 -c "import json;d=json.loads([l for l in open('$O/ab_$name.log') if l.startswith('{')][-1]);p=d['phase_ms_single_proof'];print('$name', d['value'], d['ms_per_step'], d['single_proof_latency_ms'], [p[k] for k in ('round1','round2','round3','round5')])" | tee -a $O/ab.txt
}
L=nzcb-circom_amd/lib/libnzcb.so; A=nzcb-circom_amd/lib/ab
for rep in 1 2 3; do
  run r5 $A/libnzcb_r5.so || exit $?
  run lds $L || exit $?
  run lds16 $L NZCB_SPARSE_SPAN=16 || exit $?
  run nolds $L NZCB_SPARSE_LDS=0 || exit $?
  run dense $L NZCB_SPARSE=0 || exit $?
done
echo done
