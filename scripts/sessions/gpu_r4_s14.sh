#!/bin/bash
# r4: ping-pong MX GEMM (cfg 34-36): bitwise vs cfg 24, timing on the ViT bs64 shapes; then the
# full GPU suite (executor spin, lean request path) and the single-stream latency
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_s14; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp8_gpu.py -k "pingpong or phased_bitwise or mx8_activations" > $O/pytest_mx.log 2>&1 || { tail -30 $O/pytest_mx.log; exit 1; }
tail -1 $O/pytest_mx.log
timeout -k 10 300 python3 scripts/bench_mx.py --cfgs 24,30,34,35,36 > $O/bench_mx.jsonl 2>&1 || { tail -10 $O/bench_mx.jsonl; exit 1; }
python3 -c "
import json
for l in open('$O/bench_mx.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print({k: d[k] for k in d if k != 'cfgs'}, {c: v['us'] for c, v in d['cfgs'].items()})
"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -30; exit 1; }
tail -1 $O/pytest_gpu.log
B="--steps 300 --warmup 30 --cold-trials 0 --cold-runs 0 --http-clients 0 --dp-figures 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
timeout -k 10 200 python bench.py $B > $O/bench.json 2> $O/bench_err.log || { tail -20 $O/bench_err.log; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['served_sustained']['inf_s'], d['latency_ms_p50_single'], d['latency_ms_p99_single'])"
