#!/bin/bash
set -e
o=gpurun_out/kwarg
mkdir -p $o
for i in 1 2; do
  timeout -k 10 120 ./scripts/native/conv_stamps >> $o/blockdim.jsonl 2>> $o/err.log
  timeout -k 10 120 ./scripts/native/conv_stamps_kwarg >> $o/kwarg.jsonl 2>> $o/err.log
done
timeout -k 10 400 python -u -m pytest tests/test_vision_gpu.py tests/test_engine_gpu.py tests/test_plan_gpu.py -x -q --timeout 120 --timeout-method thread > $o/test.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --cold-trials 0 --cold-runs 0 > $o/bench.json 2>> $o/err.log
