#!/bin/bash
# Round 4 window / tile-scan A/B on one box: the -m gpu suite, bench.py --steps S alternating
# the round-3 library (lib/ab/r3.so), the default (c = 17), c = 20 and the kPer = 4 scan
# variant (lib/ab/kper4.so at c = 17), then SQ_INSTS_VALU per kernel of single-lane proofs at
# c = 17 and c = 20 (collect with tools/collect_profiles.py / the summary below).
#   gpurun -- bash nzcb-circom_amd/tools/r4_ab2.sh <tag> [skip-tests] [steps]
set -o pipefail
tag=${1:-ab2}
skip=${2:-}
steps=${3:-200}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}_ab.log
: > $out
if [ -z "$skip" ]; then
  echo "== tests $(date +%T)"
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/${tag}_pytest.log; [ $rc -ne 0 ] && exit $rc
fi
R3=nzcb-circom_amd/lib/ab/r3.so
V=nzcb-circom_amd/lib/ab/kper4.so
echo "== bench $(date +%T)"
for rep in 1 2; do
  for cfg in "NZCB_LIB=$R3" "NZCB_FB_WINDOW=17" "NZCB_FB_WINDOW=20" "NZCB_LIB=$V NZCB_FB_WINDOW=17"; do
    env $cfg timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-probe --steps $steps > gpurun_out/${tag}_bench.log 2>&1 || exit $?
    echo "[$cfg] bench $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/${tag}_bench.log') if l.startswith('{')][-1]);print(d['value'], d['ms_per_step'], d['single_proof_latency_ms'])")" | tee -a $out
  done
done
echo "== valu $(date +%T)"
for w in 17 20; do
  d=gpurun_out/${tag}_pmc$w
  rm -rf $d
  NZCB_FB_WINDOW=$w timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $d -o run --output-format csv \
    -- python3 bench.py --lanes 1 --steps 4 --warmup 1 --no-cpu-baseline --no-probe > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  echo "[NZCB_FB_WINDOW=$w] VALU per proof" >> $out
  python3 - "$d" >> $out <<'PY' || exit 1
import csv, collections, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(float); n = collections.Counter()
rows = list(csv.DictReader(open(f)))
for r in rows:
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
    if r["Counter_Name"] == "SQ_INSTS_VALU":
        agg[k] += float(r["Counter_Value"]); n[k] += 1
tot = sum(agg.values())
print(f"  all kernels {tot / 1e9:.3f} G wave-VALU over the run")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:24]:
    print(f"  {k:60s} {n[k]:5d} launches {v / 1e9:8.3f} G {100 * v / tot:5.1f}%")
PY
  rm -rf $d
done
cat $out
