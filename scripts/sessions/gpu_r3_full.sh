#!/bin/bash
# the whole GPU test tier + smoke(), as the driver runs them at round end
# (optional $1: pytest -k / start file list is not used; the full tier always runs)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r3_full
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3_full/pytest.log 2>&1 || { grep -E "FAILED|ERROR|passed|failed" gpurun_out/r3_full/pytest.log | tail -30; exit 1; }
tail -15 gpurun_out/r3_full/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r3_full/smoke.log 2>&1 \
  || { tail -40 gpurun_out/r3_full/smoke.log; exit 1; }
tail -3 gpurun_out/r3_full/smoke.log
