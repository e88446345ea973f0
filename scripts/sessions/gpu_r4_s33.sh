#!/bin/bash
# r4: final full bench after the HTTP figure change (+ suite, smoke)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_s33; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -30; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench_err.log || { tail -20 $O/bench_err.log; exit 1; }
tail -1 $O/bench.json | cut -c1-1500
