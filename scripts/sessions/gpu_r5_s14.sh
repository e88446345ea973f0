#!/bin/bash
# r5 s14: fused QKV + attention (qkvatt) tests + BERT A/B (HIPZAP_QKVATT=0/1, bs16, 1 and 4
# contexts), BERT kernel stats with it; then the driver-form bench (cold start plan vs .pth after
# the rebuild) and the whole GPU suite
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s14; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_transformers_gpu.py > $O/pytest_tx.log 2>&1
echo "pytest tx rc=$?"
grep -E 'FAILED|ERROR|passed|failed' $O/pytest_tx.log | tail -10
for rep in 1 2; do
  for v in 0 1; do
    HIPZAP_QKVATT=$v timeout -k 10 200 python3 scripts/bench_models.py bert-base > $O/bert_qa${v}_$rep.jsonl 2> $O/bert_qa${v}_$rep.err || { tail -5 $O/bert_qa${v}_$rep.err; exit 1; }
    echo "qkvatt=$v rep $rep: $(python3 -c "
import json; print([(j['contexts'], j.get('items_per_s'), j.get('latency_ms_p50')) for j in map(json.loads, open('$O/bert_qa${v}_$rep.jsonl'))])")"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/pb -o run -- python3 scripts/prof_model.py --model bert-base --batch 16 --iters 20 > $O/prof_bert.log 2>&1 || { tail -20 $O/prof_bert.log; exit 1; }
db=$(find $O/pb -name '*results.db' | head -1)
python3 scripts/rocpd_stats.py "$db" 14 > $O/kernel_stats_bert_bs16.txt
rm -rf $O/pb
cut -c1-160 $O/kernel_stats_bert_bs16.txt
timeout -k 10 600 python3 bench.py > $O/bench.log 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -1 $O/bench.log > $O/bench.json
python3 -c "
import json; j=json.load(open('$O/bench.json'))
print('value', j['value'], 'ms/step', j['ms_per_step'], 'sustained', j.get('served_sustained'))
for k in ('cold_start_ms_p50','cold_start_pth_ms_p50','cold_start_pth_torch_ms_p50','cold_start_native_ms_p50','cold_start_bert_plan_ms_p50','latency_ms_p50_single'):
    print(k, j.get(k))
"
grep -i 'skipped' $O/bench.err | head -5
timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
echo "pytest rc=$?"
grep -E 'FAILED|ERROR|passed|failed' $O/pytest.log | tail -25
