#!/bin/bash
# phased 256-row MX-fp8 GEMM (cfg 46/47): bitwise vs cfg 24, then the ViT bs64 shapes
set -u
export TMPDIR=/tmp
o=gpurun_out/r3_mxk; mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp8_gpu.py \
  -k "phased or mx8_activations" > $o/pytest.log 2>&1 || { grep -E "FAILED|Error|error|passed|failed" $o/pytest.log | tail -30; exit 1; }
tail -2 $o/pytest.log
timeout -k 10 300 python -u scripts/bench_mx.py --cfgs 21,24,46,47 > $o/bench_mx.jsonl 2>&1 || { tail -20 $o/bench_mx.jsonl; exit 1; }
python3 -c "
import json
for l in open('$o/bench_mx.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], {k:v['us'] for k,v in d['cfgs'].items()})
"
