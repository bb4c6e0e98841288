#!/bin/bash
# needs a diagnostic build (not committed) for the padding: an extra
# lane creates NZCB_LANE_PAD x lane streams before its own (Prover::Prover(const Prover&, int lane))
# lane speeds by lane index, with 0..3 padding streams per lane index before each extra lane's streams
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/g; rm -rf $O; mkdir -p $O
for pad in 0 1 2 3; do
  NZCB_LANE_PAD=$pad timeout -k 10 300 rocprofv3 --marker-trace -d $O/t$pad -o run --output-format csv \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe > $O/b$pad.log 2>&1 || exit $?
  echo "== pad $pad: $(python3 -c "import json;d=json.loads([l for l in open('$O/b$pad.log') if l.startswith('{')][-1]);print(d['value'], d['ms_per_step'])")"
  python3 nzcb-circom_amd/tools/lane_speeds.py $O/t$pad 20
done
for rep in 1 2; do for pad in 0 1 2 3; do
  NZCB_LANE_PAD=$pad timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-probe > $O/b.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][-1]);print('pad$pad steps20', d['value'], d['ms_per_step'])"
done; done
