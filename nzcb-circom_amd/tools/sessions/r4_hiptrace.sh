#!/bin/bash
# HIP API + kernel + marker trace of single-lane proofs, this build and lib/ab/<variant>.so:
# which host calls block inside plonk_prove (tools/api_blocks.py reads gpurun_out/<tag>_<i>).
#   gpurun -- bash nzcb-circom_amd/tools/r4_hiptrace.sh <tag> <variant>
set -o pipefail
tag=$1; variant=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for cfg in "NZCB_R4=1" "NZCB_LIB=nzcb-circom_amd/lib/ab/${variant}.so"; do
  d=gpurun_out/${tag}_$i; rm -rf $d
  env $cfg timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --marker-trace -d $d -o run --output-format csv \
    -- python3 bench.py --lanes 1 --steps 4 --warmup 1 --no-cpu-baseline --no-probe > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  echo "[$cfg] $(ls $d/*/ 2>/dev/null | head -3 | tr '\n' ' ')"
  i=$((i + 1))
done
