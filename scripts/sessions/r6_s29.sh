#!/bin/bash
# r6 session 29: the whole GPU suite and smoke() on the final tree.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s29
mkdir -p $OUT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -n 3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -n 20; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; tail -n 2 $OUT/smoke.log; exit $rc
