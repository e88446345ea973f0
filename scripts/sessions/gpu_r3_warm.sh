#!/bin/bash
# device-code warm-up thread in hz_plan_open: plan tests, then the fresh-process plan cold start
# interleaved with HIPZAP_PLAN_CODE_WARM=0 (7 trials each, twice)
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r3_warm; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_plan_gpu.py tests/test_pth_lite_gpu.py tests/test_native_server_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 5 --warmup 2 --cold-trials 1 --dyn-batch 1 --http-clients 0 --dp-figures 0 > $O/prep.log 2>&1 || { tail -20 $O/prep.log; exit 1; }
PLAN=$(ls /tmp/hipzap_bench/*.hzplan | head -1)
for rep in 1 2; do
  for v in 1 0; do
    HIPZAP_PLAN_CODE_WARM=$v timeout -k 10 200 python -u -c "
import json; from hipzap.coldstart import measure_fresh
r = measure_fresh('plan', '$PLAN', 'resnet50', 7)
print(json.dumps({'warm': $v, 'p50': r['p50_ms'], 'all': r['all_ms'], 'phases': r['median_trial_phases_ms']}))" >> $O/cold.jsonl 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  done
done
python3 -c "
import json
for l in open('$O/cold.jsonl'):
    d=json.loads(l); p=d['phases']; print(d['warm'], d['p50'], 'hip_init', p.get('hip_init_ms'), 'upload', p.get('upload_ms'), 'first_req', round(p.get('first_request',0),2), 'total', p.get('total_ms'))"
