#!/bin/bash
# round 3: batched AWD-LSTM decode -- numerics tests, then the concurrent-request bench
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r3_lmb
timeout -k 10 400 python -u -m pytest tests/test_lmbatch_gpu.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r3_lmb/pytest.log 2>&1 || { tail -60 gpurun_out/r3_lmb/pytest.log; exit 1; }
tail -15 gpurun_out/r3_lmb/pytest.log
timeout -k 10 300 python -u scripts/bench_lm_batch.py --clients 1 8 32 64 --requests 12 --compare-pool 4 \
  > gpurun_out/r3_lmb/bench.json 2> gpurun_out/r3_lmb/bench.err || { tail -30 gpurun_out/r3_lmb/bench.err; exit 1; }
cat gpurun_out/r3_lmb/bench.json
