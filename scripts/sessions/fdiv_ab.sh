#!/bin/bash
# conv prologue division A/B (conv_stamps vs conv_stamps_intdiv), vision/engine/transformer GPU
# tests, headline bench. Binaries are built on the CPU side beforehand (hipcc, see the .hip header).
set -e
o=gpurun_out/fdiv
mkdir -p $o
for i in 1 2; do
  timeout -k 10 120 ./scripts/native/conv_stamps_intdiv >> $o/intdiv.jsonl 2>> $o/err.log
  timeout -k 10 120 ./scripts/native/conv_stamps >> $o/fdiv.jsonl 2>> $o/err.log
done
timeout -k 10 400 python -u -m pytest tests/test_vision_gpu.py tests/test_engine_gpu.py tests/test_transformers_gpu.py -x -q --timeout 120 --timeout-method thread > $o/test.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --cold-trials 0 --cold-runs 0 > $o/bench.json 2>> $o/err.log
