#!/bin/bash
# device packing of transformer linears: bitwise tests + the engines that use it + model cold starts
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r3_txpack; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_transformers_gpu.py tests/test_fp8_gpu.py tests/test_text_plan_gpu.py tests/test_pth_lite_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u scripts/bench_models.py bert-base bert-base-fp8 vit-b16-fp8 > $O/models.jsonl 2> $O/models.err || { tail -10 $O/models.err; exit 1; }
cut -c1-160 $O/models.jsonl
