#!/bin/bash
# HIP runtime pool sizes: same-box bench A/B (tools/r4_envab.sh), then a single-lane
# timeline under each setting (tools/timeline.py), to see whether launches still block.
#   gpurun -- bash nzcb-circom_amd/tools/r4_envtl.sh <tag> <steps> "<VAR=a ...>" ["<VAR=b ...>" ...]
set -o pipefail
tag=$1; steps=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash nzcb-circom_amd/tools/r4_envab.sh "$@" || exit 1
shift 2
i=0
for cfg in "$1" "${@: -1}"; do   # the first and the last setting only
  d=gpurun_out/${tag}_tl$i; rm -rf $d
  env $cfg timeout -k 10 240 rocprofv3 --kernel-trace --marker-trace -d $d -o run --output-format csv \
    -- python3 bench.py --lanes 1 --steps 6 --warmup 2 --no-cpu-baseline --no-probe > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  { echo "[$cfg]"; python3 nzcb-circom_amd/tools/timeline.py $d --proof -2 | head -8; } >> gpurun_out/${tag}.txt
  i=$((i + 1))
done
cat gpurun_out/${tag}.txt
# and, when lib/ab/q4.so is present, the quotient kernel at 4 waves per SIMD (same box)
if [ -f nzcb-circom_amd/lib/ab/q4.so ]; then
  bash nzcb-circom_amd/tools/r4_libab.sh ${tag}_q4 q4 'k_quotient' 200 || exit 1
fi
