#!/bin/bash
# Round-end rehearsal: the full GPU test suite, smoke(), then the default bench (what the driver runs).
set -e
o=${1:-gpurun_out/final}
mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_suite.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
timeout -k 10 300 python bench.py > $o/bench.json 2> $o/bench.err
