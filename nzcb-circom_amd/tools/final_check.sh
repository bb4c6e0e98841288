#!/bin/bash
# End-of-round check on one box (from the repo root, GPU box): the whole -m gpu suite, smoke(),
# the default bench.py line, and one same-box pair against the previous round's library
# (lib/ab/libnzcb_r5.so, built from round 5's last commit) at --steps 300; the pair runs twice;
# then two 2-rank rehearsals over gloo with both ranks on cuda:0 (the batch flow, and the
# single-proof MSM split with all nine commitments), when FINAL_REHEARSE=1.
#   bash nzcb-circom_amd/tools/final_check.sh   -> gpurun_out/final/{pytest,smoke,bench,ab_*}.log
# Each GPU step has its own time limit; the first failure ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
step smoke
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
step bench
timeout -k 10 600 python3 -u bench.py > $O/bench.log 2>&1 || exit $?
grep '^{"metric"' $O/bench.log | tail -1 | cut -c1-400
PREV=nzcb-circom_amd/lib/ab/libnzcb_r5.so
if [ -f $PREV ]; then
  for cfg in r6 r5 r6b r5b; do
    L=nzcb-circom_amd/lib/libnzcb.so; [ ${cfg:0:2} = r5 ] && L=$PREV
    step "ab $cfg"
    NZCB_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-probe > $O/ab_$cfg.log 2>&1 || exit $?
    python3 -c "import json;d=json.loads([l for l in open('$O/ab_$cfg.log') if l.startswith('{')][-1]);print('$cfg', d['value'], d['ms_per_step'], d['single_proof_latency_ms'])"
  done
fi
if [ "${FINAL_REHEARSE:-0}" = 1 ]; then
  step "rehearsal batch"
  NZCB_DIST_BACKEND=gloo NZCB_BENCH_DEVICE=0 timeout -k 10 400 python3 -u bench.py --gpus 2 --lanes 3 --no-cpu-baseline \
    --no-probe > $O/rehearse_batch.log 2>&1 || exit $?
  grep '^{"metric"' $O/rehearse_batch.log | tail -1 | cut -c1-300
  step "rehearsal split"
  NZCB_DIST_BACKEND=gloo NZCB_BENCH_DEVICE=0 timeout -k 10 400 python3 -u bench.py --gpus 2 --msm-split --steps 5 \
    --warmup 1 --no-cpu-baseline --no-probe > $O/rehearse_split.log 2>&1 || exit $?
  grep '^{"metric"' $O/rehearse_split.log | tail -1 | cut -c1-300
fi
step done
