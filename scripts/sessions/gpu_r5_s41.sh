#!/bin/bash
# r5 s41: LayerNorm with gamma / beta through LDS once per workgroup (HIPZAP_LN_GLDS=1) instead of
# once per wave: transformer tests under it, then interleaved A/B on BERT bs16 and the ViT
# config-5 dp figures
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s41; mkdir -p $O
HIPZAP_LN_GLDS=1 timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_transformers_gpu.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"
grep -E 'FAILED|ERROR|passed|failed' $O/pytest.log | tail -12
[ $rc -eq 0 ] || exit 1
B="--steps 5 --warmup 2 --cold-trials 0 --cold-runs 0 --http-clients 0 --dyn-batch 0 --bert-cold 0 --lm-cold 0"
for rep in 1 2; do
  for v in 0 1; do
    HIPZAP_LN_GLDS=$v timeout -k 10 200 python3 scripts/bench_models.py bert-base > $O/bert_${v}_$rep.jsonl 2> $O/bert_${v}_$rep.err || { tail -5 $O/bert_${v}_$rep.err; exit 1; }
    bert=$(python3 -c "
import json; print([(j['contexts'], j.get('items_per_s')) for j in map(json.loads, open('$O/bert_${v}_$rep.jsonl'))])")
    HIPZAP_LN_GLDS=$v timeout -k 10 300 python3 bench.py $B > $O/bench_${v}_$rep.log 2>&1 || { tail -20 $O/bench_${v}_$rep.log; exit 1; }
    vit=$(python3 -c "
import json; j=json.loads(open('$O/bench_${v}_$rep.log').read().strip().splitlines()[-1]); d=j['dp_scatter']
print(d['vit_b16_fp8_gb64']['img_s'], d['dp_shard_w8']['vit_b16_fp8_bs8']['img_s'])")
    echo "glds=$v rep $rep bert $bert vit $vit"
  done
done
