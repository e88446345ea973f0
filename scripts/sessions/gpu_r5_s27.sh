#!/bin/bash
# r5 s27: torch-free cold start with / without the interpreter's site-packages scan (python -S),
# 10 interleaved trials; then the driver-form bench with the -S workers
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s27; mkdir -p $O
python3 -c "import time; t=time.perf_counter(); import subprocess, sys, statistics
for f in ([], ['-S']):
    ts=[]
    for _ in range(10):
        t=time.perf_counter(); subprocess.run([sys.executable, *f, '-c', 'pass']); ts.append((time.perf_counter()-t)*1e3)
    print('python', f, 'start ms p50', round(statistics.median(ts), 2))"
PLAN=$(timeout -k 10 300 python3 -c "
import sys; sys.argv=['bench.py']; import bench
print(bench.prepare_artifacts('resnet50', '/tmp/hipzap_bench')[1])" 2> $O/prep.err | tail -1) || { tail -5 $O/prep.err; exit 1; }
echo "plan: $PLAN"
timeout -k 10 400 python3 scripts/cold_site_ab.py "$PLAN" --trials 10 > $O/cold_site_ab.jsonl 2> $O/cold_site_ab.err || { tail -5 $O/cold_site_ab.err; exit 1; }
tail -1 $O/cold_site_ab.jsonl
timeout -k 10 600 python3 bench.py > $O/bench.log 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -1 $O/bench.log > $O/bench.json
python3 -c "
import json; j=json.load(open('$O/bench.json'))
print('value', j['value'], 'sustained', j.get('served_sustained'))
cf=j.get('cold_start_fresh_process') or {}
for k,v in cf.items(): print(k, v.get('p50_ms'), v.get('all_ms'))
"
