#!/bin/bash
# self-launched 4-rank rehearsal on ONE GPU (gloo, ranks folded onto cuda:0) with every secondary
# figure on (sustained window, BERT plan cold start, HTTP serving through hipzap serve --gpus 2)
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r3_launch2_final
mkdir -p $O
HIPZAP_DIST_BACKEND=gloo HIPZAP_SHARE_GPU=1 timeout -k 10 900 python bench.py --gpus 2 --steps 20 --warmup 5 \
  > $O/self_launch_2.log 2>&1 || { tail -40 $O/self_launch_2.log; exit 1; }
grep '^{' $O/self_launch_2.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.readline())
print({k: d.get(k) for k in ('value','n_gpus','cold_start_ms_p50','cold_start_bert_plan_ms_p50','served_sustained')})
print('http', d.get('http_serving'))"
