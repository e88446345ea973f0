#!/bin/bash
# cold start with the torch-free children started as python -S (plus the with-site reference)
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r3_nosite; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_plan_gpu.py tests/test_pth_lite_gpu.py tests/test_text_plan_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 1; }
  grep "^{" $O/bench_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.readline()); f=d['cold_start_fresh_process']
print(d['value'], 'plan -S', d['cold_start_ms_p50'], 'plan site', d['cold_start_plan_with_site_ms_p50'], 'pth-lite', d['cold_start_pth_ms_p50'], 'bert', d['cold_start_bert_plan_ms_p50'])
print('  -S  ', f['plan']['median_trial_phases_ms'])
print('  site', f['plan_with_site']['median_trial_phases_ms'])"
done
