#!/bin/bash
# round 6: the A, B, C MSM on the real statement: entry counts / carry spans (MSMSTATS build) and
# per-kernel times with one kernel at a time (NZCB_SERIAL), sparse and dense schedules
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; O=gpurun_out/r6h; rm -rf $O; mkdir -p $O
for cfg in sparse dense; do
  E=""; [ $cfg = dense ] && E="NZCB_SPARSE=0"
  echo "== $cfg $(date +%T)"
  env NZCB_LIB=nzcb-circom_amd/lib/ab/libnzcb_stats.so NZCB_SERIAL=1 $E timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace -d $O/t_$cfg -o run --output-format csv \
    -- python3 bench.py --lanes 1 --steps 3 --warmup 1 --no-cpu-baseline --no-probe > $O/t_$cfg.log 2>&1 || exit $?
  grep MSMSTATS $O/t_$cfg.log | sort | uniq -c | sort -rn | head -12
  python3 nzcb-circom_amd/tools/timeline.py $O/t_$cfg --proof -2 > $O/timeline_$cfg.txt
  rm -rf $O/t_$cfg
done
echo done
