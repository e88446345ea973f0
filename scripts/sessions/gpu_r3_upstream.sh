#!/bin/bash
# weightless template fill on the plan's upload stream (hz_plan_upload_stream): plan / pth-lite /
# cluster tests, then fresh-process pth-lite and plan cold starts (5 trials x 2 rounds)
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r3_upstream; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_plan_gpu.py tests/test_pth_lite_gpu.py tests/test_cluster_gpu.py tests/test_text_plan_gpu.py tests/test_native_server_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u -c "
import bench, json
ck, plan = bench.prepare_artifacts('resnet50', '/tmp/hipzap_bench')
json.dump({'ckpt': ck, 'plan': plan}, open('$O/paths.json', 'w'))" > $O/prep.log 2>&1 || { tail -20 $O/prep.log; exit 1; }
for rep in 1 2; do
  timeout -k 10 300 python -u -c "
import json; from hipzap.coldstart import measure_fresh
p = json.load(open('$O/paths.json'))
for mode, path in (('pth-lite', p['ckpt']), ('plan', p['plan'])):
    r = measure_fresh(mode, path, 'resnet50', 5)
    print(json.dumps({'what': mode, 'p50': r['p50_ms'], 'all': r['all_ms'], 'phases': r['median_trial_phases_ms']}), flush=True)" >> $O/cold.jsonl 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
done
python3 -c "
import json
for l in open('$O/cold.jsonl'):
    d=json.loads(l); p=d['phases']; print(d['what'], d['p50'], d['all'], {k: p.get(k) for k in ('hip_init_ms','upload_ms','upload_raw_ms','ctx_alloc_ms','total_ms','engine_total')})"
