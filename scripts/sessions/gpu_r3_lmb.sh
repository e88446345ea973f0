#!/bin/bash
# round 3: batched AWD-LSTM decode -- numerics tests, then the concurrent-request bench (A/B of
# the layer kernel's tiles per workgroup)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r3_lmb
timeout -k 10 400 python -u -m pytest tests/test_lmbatch_gpu.py tests/test_lm_gpu.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r3_lmb/pytest.log 2>&1 || { tail -60 gpurun_out/r3_lmb/pytest.log; exit 1; }
tail -5 gpurun_out/r3_lmb/pytest.log
for tpw in 2 1 2; do
  HIPZAP_LMB_TPW=$tpw timeout -k 10 300 python -u scripts/bench_lm_batch.py --clients 1 32 64 --requests 12 \
    > gpurun_out/r3_lmb/bench_tpw$tpw.json 2> gpurun_out/r3_lmb/bench.err || { tail -30 gpurun_out/r3_lmb/bench.err; exit 1; }
  echo "tpw=$tpw"; cat gpurun_out/r3_lmb/bench_tpw$tpw.json
done
