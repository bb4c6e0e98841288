#!/bin/bash
# Round 4: the prover GPU tests, then SQ counters per kernel of single-lane proofs (where a
# kernel's time goes: VALU instructions, waves, wave cycles, waits), for the prover kernels.
#   gpurun -- bash nzcb-circom_amd/tools/r4_valu.sh <tag>
set -o pipefail
tag=${1:-valu}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}.txt
: > $out
echo "== tests $(date +%T)"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_prover.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 400 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_pytest.log; [ $rc -ne 0 ] && exit $rc
echo "== pmc $(date +%T)"
d=gpurun_out/${tag}_pmc; rm -rf $d
NZCB_SERIAL=1 timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
  SQ_INSTS_LDS SQ_ACTIVE_INST_VALU -d $d -o run --output-format csv \
  -- python3 bench.py --lanes 1 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
python3 - "$d" >> $out <<'PY' || exit 1
import csv, collections, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:44]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVES": n[k] += 1
print("# per launch: VALU = SQ_INSTS_VALU (wave instr), waves, wave-cycles, LDS instr, active-VALU and wait cycles (quad-cycles)")
for k, c in sorted(agg.items(), key=lambda kv: -kv[1]["SQ_INSTS_VALU"])[:30]:
    m = max(n[k], 1)
    print(f"  {k:44s} {n[k]:4d} x  VALU {c['SQ_INSTS_VALU']/m/1e6:8.2f} M  waves {c['SQ_WAVES']/m:9.0f}  "
          f"wave-cyc {c['SQ_WAVE_CYCLES']/m/1e6:8.2f} M  LDS {c['SQ_INSTS_LDS']/m/1e6:7.2f} M  "
          f"actVALU {c['SQ_ACTIVE_INST_VALU']/m/1e6:8.2f} M  waitInst {c['SQ_WAIT_INST_ANY']/m/1e6:8.2f} M")
PY
rm -rf $d
cat $out
