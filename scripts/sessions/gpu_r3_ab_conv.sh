#!/bin/bash
# same-box interleaved A/B: conv epilogue prefetch (new, in-tree lib) vs without (abx/libhipzap_base.so)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r3_ab_conv
mkdir -p $OUT
for rep in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export HIPZAP_LIB=hipzap/_lib/abx/libhipzap_base.so; else unset HIPZAP_LIB; fi
    timeout -k 10 200 python bench.py --steps 300 --warmup 30 --cold-trials 0 --cold-runs 0 --dyn-batch 0 > $OUT/${v}_$rep.log 2>&1 || { echo "FAIL $v"; tail -20 $OUT/${v}_$rep.log; exit 1; }
    python3 - "$OUT/${v}_$rep.log" "$v" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(sys.argv[2], d["value"], d["latency_ms_p50_single"], d["single_stream_inf_s"])
PY
  done
done
