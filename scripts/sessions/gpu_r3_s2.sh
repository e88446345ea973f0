#!/bin/bash
# Round 3 session 2 check: new GPU tests (text plans, RCCL shrink/reform, fp8, transformers),
# the driver-form bench (new secondary figures), BERT A/B vs the round-2 library.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/${TAG:-r3_s2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_text_plan_gpu.py tests/test_cluster_gpu.py tests/test_transformers_gpu.py \
  tests/test_fp8_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { grep -E "FAILED|ERROR|Error|passed|failed" $O/pytest.log | tail -30; exit 1; }
tail -3 $O/pytest.log
grep "bert plan cold start" $O/pytest.log | cut -c1-300
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.readline())
print({k: d.get(k) for k in ('value','cold_start_ms_p50','cold_start_pth_ms_p50','cold_start_bert_plan_ms_p50','served_sustained','latency_ms_p50_single')})
print('http', d.get('http_serving'))"
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export HIPZAP_LIB=hipzap/_lib/base/libhipzap_base.so; else unset HIPZAP_LIB; fi
    timeout -k 10 300 python3 scripts/bench_models.py bert-base > $O/models_${v}_$rep.jsonl 2> $O/models_${v}_$rep.err \
      || { tail -5 $O/models_${v}_$rep.err; exit 1; }
    echo "$v $rep: $(cut -c1-110 $O/models_${v}_$rep.jsonl | tr '\n' ' ')"
  done
done
echo done
