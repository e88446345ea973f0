#!/bin/bash
# persistent conv chain (HIPZAP_CONV_CHAIN): correctness, then same-box interleaved A/B vs per-conv launches
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r3_chain
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_conv_chain_gpu.py -x -v --timeout 240 --timeout-method thread \
  > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -8 $OUT/pytest.log
for rep in 1 2; do
  for v in base layer3 layer4 layer2; do
    if [ $v = base ]; then unset HIPZAP_CONV_CHAIN; else export HIPZAP_CONV_CHAIN=$v; fi
    timeout -k 10 200 python bench.py --steps 300 --warmup 30 --cold-trials 0 --cold-runs 0 --dyn-batch 0 > $OUT/${v}_$rep.log 2>&1 || { echo "FAIL $v"; tail -20 $OUT/${v}_$rep.log; exit 1; }
    python3 - "$OUT/${v}_$rep.log" "$v" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(sys.argv[2], d["value"], d["latency_ms_p50_single"], d["single_stream_inf_s"])
PY
  done
done
