#!/bin/bash
# r4: fused-kernel correctness (layer1 + layer2 bottlenecks) and stamps, before the A/B session
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_s6; mkdir -p $O
timeout -k 10 60 ./scripts/native/block_stamps > $O/stamps.jsonl 2>&1 && cat $O/stamps.jsonl || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
