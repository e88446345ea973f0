#!/bin/bash
# AWD-LSTM decode on one GPU: tests, per-kernel diag (fused sampler and tournament), bench, and a
# rocprofv3 kernel trace of the bench (in-situ kernel durations).   bash scripts/lm_profile.sh OUT
set -u
out=${1:-gpurun_out/lm}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 python -u -m pytest tests/test_lm_gpu.py -x -q --timeout 120 --timeout-method thread > "$out/test.log" 2>&1 || exit 1
timeout -k 10 120 python -u scripts/diag_lm.py > "$out/diag.json" 2>> "$out/err.log" || exit 1
HIPZAP_SAMPLER_TOURNAMENT=1 timeout -k 10 120 python -u scripts/diag_lm.py > "$out/diag_unfused.json" 2>> "$out/err.log" || exit 1
timeout -k 10 120 python -u scripts/bench_lm.py > "$out/bench.json" 2>> "$out/err.log" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- python3 scripts/bench_lm.py > "$out/bench_prof.json" 2>> "$out/err.log" || exit 1
