#!/bin/bash
# Session-5 A/B: coalesced uint8 preprocess + pool_fc 16 loads in flight (new) vs the previous build (base).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_vision_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_vision.log 2>&1 || { tail -20 gpurun_out/pytest_vision.log; exit 1; }
tail -2 gpurun_out/pytest_vision.log
for s in 1 8; do
  OUT=gpurun_out/ab_s$s CMD="python bench.py --streams $s --steps 400 --warmup 40 --cold-runs 0" REPS=3 TMO=200 bash scripts/ab_lib.sh || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --streams 1 --steps 50 --warmup 5 --cold-runs 0 > gpurun_out/rocprof.log 2>&1 || exit $?
python scripts/trace_summary.py gpurun_out/prof gpurun_out/prof_summary && rm -rf gpurun_out/prof
echo done
