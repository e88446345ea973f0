#!/bin/bash
# per-plan device-code warm-up (the translation units the plan's ops launch + the packer for a
# weightless template): plan/text/pth-lite tests, then fresh-process cold starts of the ResNet-50
# plan, the torch-free .pth path and the BERT-base text plan, interleaved with HIPZAP_PLAN_CODE_WARM=0
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r3_warm3; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_plan_gpu.py tests/test_text_plan_gpu.py tests/test_pth_lite_gpu.py tests/test_native_server_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u -c "
import bench, json
ck, plan = bench.prepare_artifacts('resnet50', '/tmp/hipzap_bench')
bp = bench.prepare_bert_plan('/tmp/hipzap_bench')
json.dump({'ckpt': ck, 'plan': plan, 'bert': bp}, open('$O/paths.json', 'w'))" > $O/prep.log 2>&1 || { tail -20 $O/prep.log; exit 1; }
for rep in 1 2; do
  for v in 1 0; do
    HIPZAP_PLAN_CODE_WARM=$v timeout -k 10 300 python -u -c "
import json; from hipzap.coldstart import measure_fresh
p = json.load(open('$O/paths.json'))
for mode, path, model in (('plan', p['plan'], 'resnet50'), ('pth-lite', p['ckpt'], 'resnet50'), ('plan', p['bert'], 'bert-base')):
    r = measure_fresh(mode, path, model, 5)
    print(json.dumps({'warm': $v, 'what': mode + ':' + model, 'p50': r['p50_ms'], 'all': r['all_ms'], 'phases': r['median_trial_phases_ms']}), flush=True)" >> $O/cold.jsonl 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  done
done
python3 -c "
import json
for l in open('$O/cold.jsonl'):
    d=json.loads(l); p=d['phases']; print(d['warm'], d['what'], d['p50'], d['all'], 'first_req', round(p.get('first_request',0),2))"
