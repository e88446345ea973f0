#!/bin/bash
# end-of-session check: full GPU test suite, smoke(), rocprofv3 kernel stats of the default bench
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 30 --warmup 3 --cold-runs 0 > gpurun_out/rocprof_s32.log 2>&1 || { tail -20 gpurun_out/rocprof_s32.log; exit 1; }
grep '^{' gpurun_out/rocprof_s32.log | cut -c1-300
python scripts/trace_summary.py gpurun_out/prof gpurun_out/prof_summary_s32 && rm -rf gpurun_out/prof
