#!/bin/bash
# would a bs16 BERT request run faster as two bs8 halves on two streams? bench_models.run at
# bs16 x {1,2} contexts and bs8 x {1,2} contexts (untuned bs8 tables), same box
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r3_bertsplit; mkdir -p $O
timeout -k 10 500 python -u -c "
import json, sys
sys.path.insert(0, 'scripts')
from bench_models import run
for rep in (1, 2):
    for b, c in ((16, 1), (8, 2), (8, 1), (16, 2)):
        r = run('bert-base', b, c, iters=200)
        r['rep'] = rep
        print(json.dumps(r), flush=True)
" > $O/runs.jsonl 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
cat $O/runs.jsonl | cut -c1-220
