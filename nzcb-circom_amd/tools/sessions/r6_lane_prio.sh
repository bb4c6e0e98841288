#!/bin/bash
# needs a diagnostic build (not committed): Prover::Prover(const Prover&, int lane) creates the lane's engine and aux streams
# with hipStreamCreateWithPriority(greatest) when lane >= NZCB_LANE_PRIO_FROM
# lane stream priorities (experiment): lanes >= k with high-priority streams; lane speeds + rates at 20 and 300 steps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/j; rm -rf $O; mkdir -p $O
for k in none 2; do
  E=""; [ $k != none ] && E="NZCB_LANE_PRIO_FROM=$k"
  env $E timeout -k 10 300 rocprofv3 --marker-trace -d $O/t$k -o run --output-format csv \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe > $O/b$k.log 2>&1 || exit $?
  echo "== prio from $k: $(python3 -c "import json;d=json.loads([l for l in open('$O/b$k.log') if l.startswith('{')][-1]);print(d['value'], d['ms_per_step'])")"
  python3 nzcb-circom_amd/tools/lane_speeds.py $O/t$k 20
done
for rep in 1 2 3; do for k in none 2 3; do
  E=""; [ $k != none ] && E="NZCB_LANE_PRIO_FROM=$k"
  env $E timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe > $O/b.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][-1]);print('prio$k steps20', d['value'], d['ms_per_step'], d['single_proof_latency_ms'])"
done; done
for k in none 2 none 2; do
  E=""; [ $k != none ] && E="NZCB_LANE_PRIO_FROM=$k"
  env $E timeout -k 10 300 python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-probe > $O/b.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][-1]);print('prio$k steps300', d['value'], d['ms_per_step'])"
done
