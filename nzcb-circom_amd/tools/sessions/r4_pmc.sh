#!/bin/bash
# Round 4 scan-kernel evidence: FETCH_SIZE and WRITE_SIZE per launch (separate --pmc passes)
# and isolated durations (NZCB_SERIAL=1 kernel trace) of the round-2 / round-5 scan kernels,
# round-3 library (lib/ab/r3.so) against this round's; then the microbenchmarks.
#   gpurun -- bash nzcb-circom_amd/tools/r4_pmc.sh <tag>
set -o pipefail
tag=${1:-pmc}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}.txt
: > $out
RX='k_perm|k_apply|k_lin|k_chunk_prod|k_scan_mul|k_shift_down|k_div_check|msm_accumulate29'
B="python3 bench.py --lanes 1 --steps 2 --warmup 1 --no-cpu-baseline --no-probe"
for cfg in "NZCB_LIB=nzcb-circom_amd/lib/ab/r3.so" "NZCB_R4=1"; do
  echo "== $cfg $(date +%T)"
  dirs=
  for c in FETCH_SIZE WRITE_SIZE; do
    d=gpurun_out/${tag}_$c; rm -rf $d
    env $cfg timeout -s KILL 240 rocprofv3 --pmc $c -d $d -o run --output-format csv -- $B > $d.log 2>&1 \
      || { tail -5 $d.log; exit 1; }
    dirs="$dirs $d"
  done
  d=gpurun_out/${tag}_trace; rm -rf $d
  env $cfg NZCB_SERIAL=1 timeout -k 10 240 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- $B > $d.log 2>&1 \
    || { tail -5 $d.log; exit 1; }
  dirs="$dirs $d"
  echo "[$cfg] per launch (FETCH_SIZE as reported: x2 for wide streaming reads on gfx950)" >> $out
  python3 nzcb-circom_amd/tools/pmc_kernels.py "$RX" $dirs >> $out || exit 1
  rm -rf $dirs
done
echo "== microbench $(date +%T)"
timeout -k 10 600 python3 nzcb-circom_amd/tools/microbench.py > gpurun_out/${tag}_micro.log 2>&1 || { tail -20 gpurun_out/${tag}_micro.log; exit 1; }
cat $out
