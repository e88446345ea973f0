#!/bin/bash
# r5 s35: round-end validation on one box: the whole GPU suite, smoke(), and the driver-form bench
# (no flags) twice
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s35; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"
grep -E 'FAILED|ERROR|passed|failed' $O/pytest.log | tail -25
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  timeout -k 10 900 python3 bench.py > $O/bench_$rep.log 2>&1 || { tail -20 $O/bench_$rep.log; exit 1; }
  tail -1 $O/bench_$rep.log > $O/bench_$rep.json
  python3 - <<PY
import json
j = json.load(open("$O/bench_$rep.json"))
d = j["dp_scatter"]
print("rep $rep value", j["value"], "ms/step", j["ms_per_step"], "sustained", j["served_sustained"]["inf_s"], "p50", j["latency_ms_p50_single"],
      "cold plan", j["cold_start_ms_p50"], "pth-lite", j.get("cold_start_pth_ms_p50"), "native", j.get("cold_start_native_ms_p50"),
      "lm", j.get("cold_start_lm_ms_p50"), "node", j.get("cold_start_node_ms_p50"), "bert", j.get("cold_start_bert_plan_ms_p50"),
      "vit64", d["vit_b16_fp8_gb64"]["img_s"], "r50gb32", d["resnet50_gb32"]["img_s"], "http", (j.get("http_serving") or {}).get("req_s"))
PY
done
