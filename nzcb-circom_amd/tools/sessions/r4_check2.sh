#!/bin/bash
# Round 4 check, second form: the -m gpu suite, bench.py (--steps S), the single-lane
# phase trace, isolated durations of the scan kernels (NZCB_SERIAL=1 kernel trace, lanes 1)
# and a c = 17 / 19 window A/B (tools/acc_probe.py + bench.py).
#   gpurun -- bash nzcb-circom_amd/tools/r4_check2.sh <tag> [skip-tests] [steps]
set -o pipefail
tag=${1:-chk}
skip=${2:-}
steps=${3:-200}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/${tag}.txt
: > $out
if [ -z "$skip" ]; then
  echo "== tests $(date +%T)"
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${tag}_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/${tag}_pytest.log; [ $rc -ne 0 ] && exit $rc
fi
line() { python3 -c "import json;d=json.loads([l for l in open('$1') if l.startswith('{')][-1]);print(d['value'], d['ms_per_step'], d['single_proof_latency_ms'], d['phase_ms_single_proof'])"; }
echo "== bench $(date +%T)"
timeout -k 10 400 python3 bench.py --steps $steps > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
echo "[default] bench $(line gpurun_out/${tag}_bench.log)" | tee -a $out
echo "== lane1 $(date +%T)"
d=gpurun_out/${tag}_lane1; rm -rf $d
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace -d $d -o run --output-format csv \
  -- python3 bench.py --lanes 1 --steps 6 --warmup 2 --no-cpu-baseline --no-probe > gpurun_out/${tag}_lane1.log 2>&1 \
  || { tail -20 gpurun_out/${tag}_lane1.log; exit 1; }
python3 nzcb-circom_amd/tools/phase_kernels.py $d > gpurun_out/${tag}_phases.txt || exit 1
rm -rf $d
echo "== serial trace $(date +%T)"
d=gpurun_out/${tag}_serial; rm -rf $d
NZCB_SERIAL=1 timeout -k 10 240 rocprofv3 --kernel-trace -d $d -o run --output-format csv \
  -- python3 bench.py --lanes 1 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
echo "[NZCB_SERIAL=1, lanes 1] scan kernels, isolated durations" >> $out
python3 nzcb-circom_amd/tools/pmc_kernels.py 'k_perm|k_apply|k_lin|k_tile_heads|k_pow_tiles|k_div_check' $d >> $out || exit 1
rm -rf $d
echo "== window $(date +%T)"
for rep in 1 2; do
  for w in 17 19; do
    r=$(NZCB_FB_WINDOW=$w timeout -k 10 120 python3 nzcb-circom_amd/tools/acc_probe.py --reps 10) || exit 1
    echo "[NZCB_FB_WINDOW=$w] acc: $r" | tee -a $out
  done
done
for w in 19 17; do
  NZCB_FB_WINDOW=$w timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-probe --steps $steps > gpurun_out/${tag}_w.log 2>&1 || exit 1
  echo "[NZCB_FB_WINDOW=$w] bench $(line gpurun_out/${tag}_w.log)" | tee -a $out
done
cat $out
