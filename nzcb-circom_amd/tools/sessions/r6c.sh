#!/bin/bash
# round 6: HIP API trace of single-lane proofs (host stalls in round 1) + same-box bench A/B vs round 5
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; O=gpurun_out/r6c; rm -rf $O; mkdir -p $O
echo "== hiptrace $(date +%T)"
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --marker-trace -d $O/ht -o run --output-format csv \
  -- python3 bench.py --lanes 1 --steps 4 --warmup 1 --no-cpu-baseline --no-probe > $O/ht.log 2>&1 || exit $?
python3 nzcb-circom_amd/tools/api_blocks.py $O/ht --min 0.05 > $O/api_blocks.txt 2>&1
head -60 $O/api_blocks.txt
rm -rf $O/ht
echo "== ab $(date +%T)"
for rep in 1 2; do
  for cfg in new r5; do
    L=nzcb-circom_amd/lib/libnzcb.so; [ $cfg = r5 ] && L=nzcb-circom_amd/lib/ab/libnzcb_r5.so
    NZCB_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-probe > $O/ab_$cfg.log 2>&1 || exit $?
    python3 -c "import json;d=json.loads([l for l in open('$O/ab_$cfg.log') if l.startswith('{')][-1]);p=d['phase_ms_single_proof'];print('$cfg', d['value'], d['ms_per_step'], d['single_proof_latency_ms'], [p[k] for k in ('round1','round2','round3','round5')])" | tee -a $O/ab.txt
  done
done
echo done
