#!/bin/bash
# r5 s33: cold-start child without argparse / pathlib / early json: the interp_to_main and
# import_lite phases of the plan and .pth-lite trials (bench.py's interleaved fresh-process runs)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s33; mkdir -p $O
B="--steps 20 --warmup 5 --http-clients 0 --dyn-batch 0 --dp-figures 0 --bert-cold 0 --lm-cold 0"
timeout -k 10 600 python3 bench.py $B > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
python3 - <<PY
import json
j = json.load(open("$O/bench.json"))
c = j["cold_start_fresh_process"]
print("value", j["value"], "plan", j["cold_start_ms_p50"], "pth_lite", j.get("cold_start_pth_ms_p50"), "native", j.get("cold_start_native_ms_p50"))
for m in ("plan", "pth_lite"):
    ph = c[m]["median_trial_phases_ms"]
    print(m, c[m]["p50_ms"], {k: ph.get(k) for k in ("spawn_to_interp", "interp_to_main", "import_lite", "hip_init_ms", "upload_ms", "stream_ms", "total_ms")})
PY
