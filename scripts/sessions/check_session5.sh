#!/bin/bash
# session-5 check: engine GPU tests, smoke(), default bench (no flags), default bench with cold-start reps
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_engine.log 2>&1 || { tail -30 gpurun_out/pytest_engine.log; exit 1; }
tail -1 gpurun_out/pytest_engine.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
grep '^{' gpurun_out/bench_default.log > gpurun_out/bench_default.json
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --cold-runs 3 > gpurun_out/bench_s32_cold.log 2>&1 || { tail -20 gpurun_out/bench_s32_cold.log; exit 1; }
grep '^{' gpurun_out/bench_s32_cold.log > gpurun_out/bench_s32_cold.json
cat gpurun_out/bench_default.json gpurun_out/bench_s32_cold.json
