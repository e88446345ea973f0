#!/bin/bash
# r6 session 5: config figures with process-based LM HTTP clients; BERT 4-context fused vs unfused
# QKV+attention; the bench's 2-rank path rehearsed on one GPU (gloo, ranks folded onto cuda:0).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s5
mkdir -p $OUT
timeout -k 10 300 python3 scripts/bench_configs.py --device 0 > $OUT/configs.log 2>&1
rc=$?; echo "configs rc=$rc"; grep '^{' $OUT/configs.log | cut -c1-3500; [ $rc -eq 0 ] || exit $rc
for q in 1 0; do
  HIPZAP_QKVATT=$q timeout -k 10 200 python3 scripts/bench_models.py bert-base > $OUT/bert_qkvatt$q.log 2>&1
  rc=$?; echo "bert qkvatt=$q rc=$rc"; grep '^{' $OUT/bert_qkvatt$q.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
HIPZAP_DIST_BACKEND=gloo HIPZAP_SHARE_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 > $OUT/rehearse_dp2.log 2>&1
rc=$?; echo "rehearse dp2 rc=$rc"; grep '^{' $OUT/rehearse_dp2.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('n_gpus', d['n_gpus'], 'value', d['value'], 'rccl_mapped', d['rccl_mapped'], 'configs', list((d.get('configs') or {}).keys()), 'http', (d.get('http_serving') or {}).get('req_per_s'), 'dp', {k: (v or {}).get('img_s') if isinstance(v, dict) else v for k, v in (d.get('dp_scatter') or {}).items()})"
[ $rc -eq 0 ] || tail -30 $OUT/rehearse_dp2.log
