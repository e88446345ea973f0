#!/bin/bash
# r4: GPU suite after the one-request LM program and the planner check; 2-rank rehearsal of the
# driver's multi-GPU bench launch (gloo, both ranks on the one GPU); LM one-client kernel stats
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4_s21; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -30; exit 1; }
tail -1 $O/pytest_gpu.log
HIPZAP_DIST_BACKEND=gloo HIPZAP_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 100 --warmup 10 > $O/rehearse_dp2.log 2>&1 || { tail -30 $O/rehearse_dp2.log; exit 1; }
grep '^{' $O/rehearse_dp2.log > $O/rehearse_dp2.json && tail -c 600 $O/rehearse_dp2.json; echo
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/lmc1 -o run -- python3 scripts/bench_lm_batch.py --clients 1 --requests 6 > $O/lmc1.log 2>&1 || { tail -20 $O/lmc1.log; exit 1; }
echo done
