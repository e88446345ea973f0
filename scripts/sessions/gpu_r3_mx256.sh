#!/bin/bash
# Round 3: pipelined 256-row MX fp8 GEMM -- correctness (bitwise vs the 128x128 kernel, fp32
# oracle), ViT-fp8 bs64 re-tune with the new tiles as candidates, config-5 bench before/after.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/${TAG:-r3_mx256}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 bench.py --mode scatter --model vit-b16-fp8 --global-batch 64 --steps 50 --warmup 5 \
  --cold-trials 0 --cold-runs 0 > $O/vit64_old.log 2>&1 || { tail -5 $O/vit64_old.log; exit 1; }
cp hipzap/tuning/vit-b16-fp8_bs64.json $O/tune_old.json
timeout -k 10 400 python -u -m hipzap.engine.tune --model vit-b16-fp8 --batch 64 --report $O/tune_report.json > $O/tune.log 2>&1 \
  || { tail -20 $O/tune.log; exit 1; }
cp hipzap/tuning/vit-b16-fp8_bs64.json $O/tune_new.json
timeout -k 10 300 python3 bench.py --mode scatter --model vit-b16-fp8 --global-batch 64 --steps 50 --warmup 5 \
  --cold-trials 0 --cold-runs 0 > $O/vit64_new.log 2>&1 || { tail -5 $O/vit64_new.log; exit 1; }
grep -h '^{' $O/vit64_old.log $O/vit64_new.log | cut -c1-160
echo done
