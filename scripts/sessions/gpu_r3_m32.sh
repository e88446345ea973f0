#!/bin/bash
# 32x32x16-MFMA LDS GEMM tiles: numerics (row-major + implicit-GEMM conv) then the GEMM microbench
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r3_m32b
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_transformers_gpu.py \
  tests/test_conv_lds_gpu.py -k "lds_gemm or conv_lds or lds_conv" > gpurun_out/r3_m32b/pytest.log 2>&1 \
  || { grep -E "FAILED|Error|error|passed|failed" gpurun_out/r3_m32b/pytest.log | tail -30; exit 1; }
tail -2 gpurun_out/r3_m32b/pytest.log
timeout -k 10 400 python -u scripts/bench_gemm.py > gpurun_out/r3_m32b/gemm.jsonl 2>&1 || { tail -20 gpurun_out/r3_m32b/gemm.jsonl; exit 1; }
cut -c1-330 gpurun_out/r3_m32b/gemm.jsonl
