#!/bin/bash
# r6 session 23: the role-split MX GEMM (cfg 40 / 41): bitwise tests vs cfg 24, then the ViT-B/16
# gb64 shapes (M = 12608) timed for cfg 24 / 30 / 40 / 41.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r6_s23
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp8_gpu.py -k "mx" > $OUT/tests.log 2>&1
rc=$?; tail -n 5 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/tests.log | head -n 20; exit $rc; }
timeout -k 10 300 python3 -u scripts/bench_mx.py --cfgs 24,40,41,42 > $OUT/bench_mx.jsonl 2> $OUT/bench_mx.err
rc=$?; cat $OUT/bench_mx.jsonl | cut -c1-400; [ $rc -eq 0 ] || { tail -n 5 $OUT/bench_mx.err; exit $rc; }
