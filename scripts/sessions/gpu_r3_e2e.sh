#!/bin/bash
# GET /inference end to end (server + Lambda) and the tightened oracles
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r3_e2e
timeout -k 10 600 python -u -m pytest tests/test_inference_e2e_gpu.py tests/test_fp8_gpu.py tests/test_transformers_gpu.py tests/test_cluster_gpu.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3_e2e/pytest.log 2>&1 || { tail -80 gpurun_out/r3_e2e/pytest.log; exit 1; }
tail -40 gpurun_out/r3_e2e/pytest.log
