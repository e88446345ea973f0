#!/bin/bash
# batched decode: tests, bench, kernel profile
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3_lmb2
timeout -k 10 300 python -u -m pytest tests/test_lmbatch_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r3_lmb2/pytest.log 2>&1 || { tail -60 gpurun_out/r3_lmb2/pytest.log; exit 1; }
tail -2 gpurun_out/r3_lmb2/pytest.log
timeout -k 10 300 python -u scripts/bench_lm_batch.py --clients 1 32 64 --requests 12 \
  > gpurun_out/r3_lmb2/bench.json 2> gpurun_out/r3_lmb2/bench.err || { tail -30 gpurun_out/r3_lmb2/bench.err; exit 1; }
cat gpurun_out/r3_lmb2/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_lmb2/prof -o run -- python3 scripts/bench_lm_batch.py --clients 32 --requests 4 > gpurun_out/r3_lmb2/prof.log 2>&1 || { tail -30 gpurun_out/r3_lmb2/prof.log; exit 1; }
db=$(find gpurun_out/r3_lmb2/prof -name '*results.db' | head -1)
python3 scripts/rocpd_stats.py "$db" 6 > gpurun_out/r3_lmb2/kernel_stats.txt
cat gpurun_out/r3_lmb2/kernel_stats.txt
rm -f "$db"
