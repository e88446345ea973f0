#!/bin/bash
# r4: serving soak -- `python -m hipzap serve` (native HTTP front end, plan image, 8 contexts) under
# 16 client processes for ~100 s (1.28 M requests): errors, rate and latency at the end of the run
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_s31; mkdir -p $O
timeout -k 10 400 python scripts/http_load.py --clients 16 --requests 80000 --format npy --server-log $O/server.log > $O/soak.json 2> $O/soak_err.log || { tail -20 $O/soak_err.log; tail -20 $O/server.log; exit 1; }
tail -c 1500 $O/soak.json
