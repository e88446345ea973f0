# HSA_ENABLE_SDMA=0 vs default: bare HIP init (probe) and the full plan cold start, interleaved
o=gpurun_out/sdma; mkdir -p $o
for t in $(seq 1 12); do
  timeout -k 5 30 ./scripts/native/hip_init_probe > $o/t.json 2>/dev/null || exit 1
  echo "{\"env\": \"base\", \"r\": $(cat $o/t.json)}" >> $o/probe.jsonl
  HSA_ENABLE_SDMA=0 timeout -k 5 30 ./scripts/native/hip_init_probe > $o/t.json 2>/dev/null || exit 1
  echo "{\"env\": \"sdma0\", \"r\": $(cat $o/t.json)}" >> $o/probe.jsonl
done
timeout -k 10 300 python -u - > $o/plan_cold.jsonl 2> $o/plan_cold.err <<'PY' || exit 2
import json, os, sys
sys.path.insert(0, ".")
from bench import prepare_artifacts
from hipzap.coldstart import measure_fresh
_, plan = prepare_artifacts("resnet50", "/tmp/hipzap_bench")
base = dict(os.environ)
sd = dict(os.environ, HSA_ENABLE_SDMA="0")
res = {"base": [], "sdma0": []}
for _ in range(9):
    res["base"].append(measure_fresh("plan", plan, trials=1, env=base))
    res["sdma0"].append(measure_fresh("plan", plan, trials=1, env=sd))
for m, rs in res.items():
    w = sorted(r["p50_ms"] for r in rs)
    med = sorted(rs, key=lambda r: r["p50_ms"])[len(rs) // 2]
    print(json.dumps({"env": m, "p50_ms": w[len(w) // 2], "all": w, "median_phases": med["median_trial_phases_ms"]}))
PY
