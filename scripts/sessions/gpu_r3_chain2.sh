#!/bin/bash
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r3_chain
mkdir -p $OUT
PYTHONPATH=. timeout -k 10 300 python -u scripts/diag_chain.py layer3:128 layer3:256 layer3:64 layer3:256:0 layer3:256:6 layer4:128 layer4:256 \
  > $OUT/diag.jsonl 2> $OUT/diag.err || { tail -30 $OUT/diag.err; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r3_chain/diag.jsonl"):
    d = json.loads(l)
    print(d["config"], d["us_per_replay"], d.get("delta_us"), d.get("chain_us_traced"), d.get("err"))
    for r in d.get("stages", []):
        print("   ", r)
PY
