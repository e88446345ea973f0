#!/bin/bash
# r5 s46: one more driver-form bench (no flags) on the final tree, another box
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s46; mkdir -p $O
timeout -k 10 900 python3 bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
python3 - <<PY
import json
j = json.load(open("$O/bench.json")); d = j["dp_scatter"]
print("value", j["value"], "sustained", j["served_sustained"]["inf_s"], "p50", j["latency_ms_p50_single"], "plan", j["cold_start_ms_p50"],
      "pth-lite", j.get("cold_start_pth_ms_p50"), "native", j.get("cold_start_native_ms_p50"), "lm", j.get("cold_start_lm_ms_p50"),
      "vit64", d["vit_b16_fp8_gb64"]["img_s"], "r50gb32", d["resnet50_gb32"]["img_s"])
PY
