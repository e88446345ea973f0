#!/bin/bash
# r6 session 6: cold-start trials back to back vs with an idle gap before each (HIPZAP_COLD_GAP_MS),
# interleaved sets, everything else off.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s6
mkdir -p $OUT
B="python3 bench.py --cold-trials 15 --lm-cold 0 --bert-cold 0 --dyn-batch 0 --http-clients 0 --dp-figures 0 --config-figures 0 --cold-runs 0 --steps 5 --warmup 2 --sustained-s 0"
for rep in 1 2; do
  for gap in 0 300; do
    HIPZAP_COLD_GAP_MS=$gap timeout -k 10 300 $B > $OUT/gap${gap}_rep$rep.log 2>&1
    rc=$?; echo "gap=$gap rep=$rep rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/gap${gap}_rep$rep.log; exit $rc; }
    grep '^{' $OUT/gap${gap}_rep$rep.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); f=d['cold_start_fresh_process']
print(' ', {k: (f[k]['p50_ms'], f[k].get('hip_init_ms_p50'), f[k].get('own_ms_p50')) for k in ('plan','pth_lite','native','pth') if isinstance(f.get(k), dict) and 'p50_ms' in f[k]})"
  done
done
