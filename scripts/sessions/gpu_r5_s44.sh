#!/bin/bash
# r5 s44: cfg 62 = the persistent tile with its MFMAs issued before the next stage's staging (branch-free step):
# persistent 256 x 256 MX-fp8 tile (one 8-wave workgroup per CU walking tiles,
# register-staged stages): bitwise vs cfg 24 (incl. 300 tiles: workgroups walk two), oracle
# tests, ViT bs64 microbench against cfg 24 / 21
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s44; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_fp8_gpu.py -k "mx8_activations or mx256" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"
grep -E 'FAILED|ERROR|passed|failed' $O/pytest.log | tail -12
[ $rc -eq 0 ] || exit 1  # any failure (a fault shows up as failures too): nothing more on the GPU
timeout -k 10 300 python3 scripts/bench_mx.py --cfgs 24,21,62 > $O/mx.jsonl 2> $O/mx.err || { tail -5 $O/mx.err; exit 1; }
python3 -c "
import json
for l in open('$O/mx.jsonl'):
    if l.startswith('{'):
        j = json.loads(l); print(j['shape'], j['best_cfg'], {c: (v['us'], v['tflops']) for c, v in j['cfgs'].items()})"
