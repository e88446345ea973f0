#!/bin/bash
# r6 session 22: the round-end checks on the final tree -- whole GPU suite, smoke(), the default
# full bench twice.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s22
mkdir -p $OUT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -n 3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -n 20; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; tail -n 2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 600 python3 bench.py > $OUT/bench_full_$rep.log 2>&1
  rc=$?; echo "bench rep $rep rc=$rc"; [ $rc -eq 0 ] || { tail -n 20 $OUT/bench_full_$rep.log; exit $rc; }
  grep '^{' $OUT/bench_full_$rep.log > $OUT/bench_full_$rep.json
  python3 - $OUT/bench_full_$rep.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); dp = d.get("dp_scatter") or {}; sh = dp.get("dp_shard_w8") or {}; c = d.get("configs") or {}
print("value", d["value"], "sustained", (d.get("served_sustained") or {}).get("inf_s"), "p50load", d.get("latency_ms_under_load_p50"),
      "cold", d.get("cold_start_ms_p50"), "b2b", d.get("cold_start_back_to_back_ms_p50"), "pth", d.get("cold_start_pth_ms_p50"),
      "native", d.get("cold_start_native_ms_p50"), "lm_cold", d.get("cold_start_lm_ms_p50"), "node", d.get("cold_start_node_ms_p50"),
      "bert_cold", d.get("cold_start_bert_plan_ms_p50"))
print("dyn", (d.get("dynamic_batching") or {}).get("inf_s"), "http", (d.get("http_serving") or {}).get("req_per_s"),
      "gb32", (dp.get("resnet50_gb32") or {}).get("img_s"), "vit", (dp.get("vit_b16_fp8_gb64") or {}).get("img_s"),
      "bs4", (sh.get("resnet50_bs4") or {}).get("img_s_in_flight"), "vit8", (sh.get("vit_b16_fp8_bs8") or {}).get("img_s_in_flight"))
b = c.get("bert_base_bs16") or {}; lm = c.get("awd_lstm_get_inference_http") or {}
print("bert", b.get("seq_s_1ctx"), b.get("seq_s_4ctx"), "lm_http", lm.get("lone_request_ms_p50"), lm.get("concurrent_req_s"))
PY
done
