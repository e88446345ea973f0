#!/bin/bash
# r5 s20: LayerNorm sized to D (2 chunks per lane at 768: 70-136 VGPRs instead of 174) and 1 / 2 / 4
# rows per wave: transformer tests, then BERT-base bs16 and ViT-B/16 fp8 bs64 per variant
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s20; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_transformers_gpu.py > $O/pytest_tx.log 2>&1
echo "pytest tx rc=$?"
grep -E 'FAILED|ERROR|passed|failed' $O/pytest_tx.log | tail -10
for rep in 1 2; do
  for r in 1 2 4; do
    HIPZAP_LN_RPW=$r timeout -k 10 300 python3 -c "
import json, sys
sys.path.insert(0, 'scripts')
from bench_models import run
for name, b in (('bert-base', 16), ('vit-b16-fp8', 64)):
    res = run(name, b, 1, iters=60)
    print(json.dumps({'rpw': $r, 'rep': $rep, 'model': name, 'batch': b, 'items_per_s': res['items_per_s'], 'p50_ms': res['latency_ms_p50']}))
" >> $O/ln_ab.jsonl 2> $O/ln_ab_${r}_$rep.err || { tail -5 $O/ln_ab_${r}_$rep.err; exit 1; }
  done
done
cat $O/ln_ab.jsonl
