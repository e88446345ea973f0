#!/bin/bash
# r5 s13: the driver-form bench (no flags) with the round-5 defaults (seam + kconv + tail): value vs
# sustained, cold-start plan vs .pth in the same run
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s13; mkdir -p $O
timeout -k 10 1000 python3 bench.py > $O/bench.log 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -1 $O/bench.log > $O/bench.json
python3 -c "
import json; j=json.load(open('$O/bench.json'))
print('value', j['value'], 'ms/step', j['ms_per_step'], 'sustained', j.get('served_sustained'))
for k in ('cold_start_ms_p50','cold_start_pth_ms_p50','cold_start_pth_torch_ms_p50','cold_start_native_ms_p50','latency_ms_p50_single'):
    print(k, j.get(k))
cf=j.get('cold_start_fresh_process') or {}
print(json.dumps(cf)[:1500])
"
