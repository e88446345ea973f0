#!/bin/bash
# r5 s25: register-ring MX-fp8 tiles (cfg 48-50): bitwise vs cfg 24 + oracle tests, then the ViT bs64
# shapes microbenchmark against cfg 24 / 21
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s25; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_fp8_gpu.py -k "mx8_activations or mx256" > $O/pytest.log 2>&1
echo "pytest rc=$?"
grep -E 'FAILED|ERROR|passed|failed' $O/pytest.log | tail -12
timeout -k 10 300 python3 scripts/bench_mx.py --cfgs 24,21,48,49,50 > $O/mx.jsonl 2> $O/mx.err || { tail -5 $O/mx.err; exit 1; }
python3 -c "
import json
for l in open('$O/mx.jsonl'):
    if l.startswith('{'):
        j = json.loads(l); print(j['shape'], j['best_cfg'], {c: v['us'] for c, v in j['cfgs'].items()})"
