#!/bin/bash
# r6 session 8: selftest (DPPipeline on the RCCL communicator at world 1), BERT seq/s against the
# timed window, the default full bench (DP figures with steps in flight), then the cold-start gap A/B.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s8
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rccl_multi_gpu.py tests/test_dp_gpu.py > $OUT/test_rccl_dp.log 2>&1
rc=$?; tail -12 $OUT/test_rccl_dp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/diag_bert_iters.py > $OUT/bert_iters.jsonl 2>$OUT/bert_iters.err
rc=$?; cat $OUT/bert_iters.jsonl; [ $rc -eq 0 ] || { tail -5 $OUT/bert_iters.err; exit $rc; }
timeout -k 10 600 python3 bench.py > $OUT/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_full.log; exit $rc; }
grep '^{' $OUT/bench_full.log > $OUT/bench_full.json
python3 -c "
import json; d=json.load(open('$OUT/bench_full.json'))
print('value', d['value'], 'cold', d.get('cold_start_ms_p50'), 'dp', json.dumps(d.get('dp_scatter'))[:1200])"
bash scripts/sessions/r6_s6.sh
