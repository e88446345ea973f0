#!/bin/bash
# r4: HTTP serving figure -- request contexts per GPU in the server (bench uses 8 with 12 clients)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_s32; mkdir -p $O
for rep in 1 2; do
  for v in 12:8 16:16 24:16 24:24; do
    cl=${v%%:*}; cx=${v##*:}
    timeout -k 10 300 python scripts/http_load.py --clients $cl --contexts $cx --requests 1500 --format npy > $O/h_${cl}_${cx}_$rep.json 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/h_${cl}_${cx}_$rep.json').read().strip().splitlines()[-1]); print('clients=$cl contexts=$cx', d['req_per_s'], d['p50_ms'], d['p99_ms'], d['errors'])"
  done
done
