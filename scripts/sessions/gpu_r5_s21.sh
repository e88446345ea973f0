#!/bin/bash
# r5 s21: full GPU suite + the driver-form bench after the round-5 changes (LN resize, xseam default, interleaved cold start)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s21; mkdir -p $O
timeout -k 10 600 python3 bench.py > $O/bench.log 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -1 $O/bench.log > $O/bench.json
python3 -c "
import json; j=json.load(open('$O/bench.json'))
print('value', j['value'], 'ms/step', j['ms_per_step'], 'sustained', j.get('served_sustained'))
print('dp', json.dumps(j.get('dp_scatter'))[:600]); print('shard', json.dumps(j.get('dp_shard_w8'))[:400])
for k in ('cold_start_ms_p50','cold_start_pth_ms_p50','cold_start_pth_torch_ms_p50','cold_start_native_ms_p50','cold_start_bert_plan_ms_p50','latency_ms_p50_single'):
    print(k, j.get(k))
"
grep -i 'skipped' $O/bench.err | head -5
timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
echo "pytest rc=$?"
grep -E 'FAILED|ERROR|passed|failed' $O/pytest.log | tail -25

