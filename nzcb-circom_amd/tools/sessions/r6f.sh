#!/bin/bash
# round 6: A, B, C in one MSM schedule (msm_enqueue_sets): parity, timeline, same-box A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; O=gpurun_out/r6f; rm -rf $O; mkdir -p $O
echo "== pytest $(date +%T)"
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_prover.py -m gpu -x -v \
  --timeout 800 --timeout-method thread -p no:cacheprovider -k "golden or prove or quotient or guard" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== lane1 $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace -d $O/t_new -o run --output-format csv \
  -- python3 bench.py --lanes 1 --steps 6 --warmup 2 --no-cpu-baseline --no-probe > $O/t_new.log 2>&1 || exit $?
python3 nzcb-circom_amd/tools/timeline.py $O/t_new --proof -2 > $O/timeline_new.txt
python3 nzcb-circom_amd/tools/phase_kernels.py $O/t_new > $O/phases_new.txt
rm -rf $O/t_new
head -30 $O/phases_new.txt
echo "== ab $(date +%T)"
run() {  # name lib env...
  local name=$1 lib=$2; shift 2
  env NZCB_LIB=$lib "$@" timeout -k 10 300 python3 -u bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-probe > $O/ab_$name.log 2>&1 || return $?
  python3 -c "import json;d=json.loads([l for l in open('$O/ab_$name.log') if l.startswith('{')][-1]);p=d['phase_ms_single_proof'];print('$name', d['value'], d['ms_per_step'], d['single_proof_latency_ms'], [p[k] for k in ('round1','round2','round3','round5')])" | tee -a $O/ab.txt
}
L=nzcb-circom_amd/lib/libnzcb.so; A=nzcb-circom_amd/lib/ab
for rep in 1 2; do
  run r5 $A/libnzcb_r5.so || exit $?
  run sets $L || exit $?
  run sets_dense $L NZCB_SPARSE=0 || exit $?
  run three $L NZCB_ABC_SETS=0 || exit $?
done
echo done
