#!/bin/bash
# r6 session 17: the default full bench twice (the driver's command), for the record.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s17
mkdir -p $OUT
for rep in 1 2; do
  timeout -k 10 600 python3 bench.py > $OUT/bench_full_$rep.log 2>&1
  rc=$?; echo "bench rep $rep rc=$rc"; [ $rc -eq 0 ] || { tail -n 20 $OUT/bench_full_$rep.log; exit $rc; }
  grep '^{' $OUT/bench_full_$rep.log > $OUT/bench_full_$rep.json
  python3 - $OUT/bench_full_$rep.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); dp = d.get("dp_scatter") or {}; sh = dp.get("dp_shard_w8") or {}; c = d.get("configs") or {}
print("value", d["value"], "cold", d.get("cold_start_ms_p50"), "b2b", d.get("cold_start_back_to_back_ms_p50"),
      "pth", d.get("cold_start_pth_ms_p50"), "native", d.get("cold_start_native_ms_p50"), "lm_cold", d.get("cold_start_lm_ms_p50"))
print("dyn", (d.get("dynamic_batching") or {}).get("inf_s"), "http", (d.get("http_serving") or {}).get("req_per_s"),
      "gb32", (dp.get("resnet50_gb32") or {}).get("img_s"), "vit", (dp.get("vit_b16_fp8_gb64") or {}).get("img_s"),
      "bs4", (sh.get("resnet50_bs4") or {}).get("img_s_in_flight"), "vit8", (sh.get("vit_b16_fp8_bs8") or {}).get("img_s_in_flight"))
b = c.get("bert_base_bs16") or {}; lm = c.get("awd_lstm_get_inference_http") or {}; lw = c.get("awd_lstm_get_inference") or {}
print("bert", b.get("seq_s_1ctx"), b.get("seq_s_4ctx"), "lm_http", lm.get("lone_request_ms_p50"), lm.get("concurrent_req_s"),
      "lm_wsgi", lw.get("lone_request_ms_p50"), lw.get("concurrent_req_s"), "plumbing", json.dumps(c.get("resnet18_cpu_plumbing"))[:200])
PY
done
