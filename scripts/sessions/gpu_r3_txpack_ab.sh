#!/bin/bash
# A/B of the device linear packing on the model cold starts (interleaved, 2 runs each)
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r3_txpack_ab; mkdir -p $O
for v in 1 0 1 0; do
  HIPZAP_NATIVE_PACK=$v timeout -k 10 300 python -u scripts/bench_models.py bert-base vit-b16-fp8 >> $O/b_$v.jsonl 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
done
for v in 1 0; do echo "NATIVE_PACK=$v"; python3 -c "
import json
for l in open('$O/b_$v.jsonl'):
    d=json.loads(l); print(' ', d['model'], d['contexts'], d['cold_start_ms'], d['items_per_s'])"; done
