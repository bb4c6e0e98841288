#!/bin/bash
# Wave-level VALU instructions per launch of each MSM kernel (tools/acc_probe.py, one
# fixed-base MSM at 2^21 + 6), one PMC pass per environment setting:
#   gpurun -- bash nzcb-circom_amd/tools/valu_probe.sh <tag> "<VAR=a ...>" ["<VAR=b ...>" ...]
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}_valu.txt
: > $out
i=0
for cfg in "$@"; do
  d=gpurun_out/${tag}_valu$i
  rm -rf $d
  env $cfg timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $d -o run --output-format csv \
    -- python3 nzcb-circom_amd/tools/acc_probe.py --reps 2 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  echo "[$cfg]" >> $out
  python3 - "$d" >> $out <<'PY' || exit 1
import csv, collections, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVES": n[k] += 1
tot = 0.0
for k, c in sorted(agg.items(), key=lambda kv: -kv[1]["SQ_INSTS_VALU"]):
    if "msm" not in k: continue
    v = c["SQ_INSTS_VALU"] / max(n[k], 1); tot += v
    print(f"  {k:60s} {n[k]:4d} launches {v / 1e6:10.2f} M VALU/launch")
print(f"  {'all msm kernels':60s} {'':14s} {tot / 1e6:10.2f} M VALU/launch")
PY
  rm -rf $d
  i=$((i + 1))
done
cat $out
