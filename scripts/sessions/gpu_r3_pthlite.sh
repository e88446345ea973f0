#!/bin/bash
# torch-free .pth cold start: GPU tests, then the bench's cold-start section (steps small)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r3_pthlite
timeout -k 10 300 python -u -m pytest tests/test_pth_lite_gpu.py tests/test_plan_gpu.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r3_pthlite/pytest.log 2>&1 || { tail -60 gpurun_out/r3_pthlite/pytest.log; exit 1; }
tail -12 gpurun_out/r3_pthlite/pytest.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_pthlite/bench.log 2>&1 || { tail -30 gpurun_out/r3_pthlite/bench.log; exit 1; }
grep '^{' gpurun_out/r3_pthlite/bench.log > gpurun_out/r3_pthlite/bench.json
python - <<'PY'
import json
d = json.load(open("gpurun_out/r3_pthlite/bench.json"))
print({k: d[k] for k in ("value", "cold_start_ms_p50", "cold_start_pth_ms_p50", "cold_start_pth_torch_ms_p50")})
print(json.dumps(d["cold_start_fresh_process"].get("pth_lite")))
PY
