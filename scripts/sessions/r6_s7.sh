#!/bin/bash
# r6 session 7: DP steps in flight (DPPipeline): its GPU test, the batched programs with C contexts
# concurrently (Engine.bench), and bench.py's configs 3 / 5 figures at HIPZAP_DP_DEPTH 1..4.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s7
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_dp_gpu.py > $OUT/test_dp_gpu.log 2>&1
rc=$?; tail -8 $OUT/test_dp_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u scripts/diag_batch_ctx.py --batches 4,8,16,32 --contexts 1,2,3,4 > $OUT/batch_ctx.jsonl 2>$OUT/batch_ctx.err
rc=$?; cat $OUT/batch_ctx.jsonl; [ $rc -eq 0 ] || { tail -5 $OUT/batch_ctx.err; exit $rc; }
B="python3 bench.py --cold-trials 0 --lm-cold 0 --bert-cold 0 --dyn-batch 0 --http-clients 0 --dp-figures 1 --config-figures 0 --cold-runs 0 --steps 40 --warmup 5 --sustained-s 0"
for d in 2 3 4; do
  HIPZAP_DP_DEPTH=$d timeout -k 10 400 $B > $OUT/dp_depth$d.log 2>&1
  rc=$?; echo "depth=$d rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/dp_depth$d.log; exit $rc; }
  grep '^{' $OUT/dp_depth$d.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); f=d.get('dp_scatter') or d.get('dp') or {}
print(' value', d['value'], json.dumps(f)[:1500])"
done
