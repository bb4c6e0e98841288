#!/bin/bash
# Same-box A/B of this build against lib/ab/<variant>.so: isolated durations of the kernels
# matching <regex> (NZCB_SERIAL=1 kernel trace, lanes 1) and bench.py --steps S, alternated.
#   gpurun -- bash nzcb-circom_amd/tools/r4_libab.sh <tag> <variant> <regex> [steps]
set -o pipefail
tag=$1; variant=$2; rx=$3; steps=${4:-200}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}.txt
: > $out
V=nzcb-circom_amd/lib/ab/${variant}.so
for cfg in "NZCB_R4=1" "NZCB_LIB=$V"; do
  d=gpurun_out/${tag}_serial; rm -rf $d
  env $cfg NZCB_SERIAL=1 timeout -k 10 240 rocprofv3 --kernel-trace -d $d -o run --output-format csv \
    -- python3 bench.py --lanes 1 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  echo "[$cfg] isolated" >> $out
  python3 nzcb-circom_amd/tools/pmc_kernels.py "$rx" $d >> $out || exit 1
  rm -rf $d
done
line() { python3 -c "import json;d=json.loads([l for l in open('$1') if l.startswith('{')][-1]);print(d['value'], d['ms_per_step'], d['single_proof_latency_ms'])"; }
for rep in 1 2; do
  for cfg in "NZCB_R4=1" "NZCB_LIB=$V"; do
    env $cfg timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-probe --steps $steps > gpurun_out/${tag}_bench.log 2>&1 || exit 1
    echo "[$cfg] bench $(line gpurun_out/${tag}_bench.log)" | tee -a $out
  done
done
cat $out
