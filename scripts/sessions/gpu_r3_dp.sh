#!/bin/bash
# DP scatter/gather figures inside bench.py (BASELINE configs 3 and 5): tune the ViT-fp8 shard
# batches the 2- and 4-rank launches use, then the driver's N=1 form and a self-launched 2-rank
# rehearsal on one GPU (gloo)
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r3_dp; mkdir -p $O/tuning
timeout -k 10 400 python -u -m hipzap tune --model vit-b16-fp8 --batch 32 16 --concurrent 1 > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
cp hipzap/tuning/vit-b16-fp8_bs32.json hipzap/tuning/vit-b16-fp8_bs16.json $O/tuning/
tail -3 $O/tune.log
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_n1.log 2>&1 || { tail -30 $O/bench_n1.log; exit 1; }
grep '^{' $O/bench_n1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d.get('dp_scatter'))"
HIPZAP_DIST_BACKEND=gloo HIPZAP_SHARE_GPU=1 timeout -k 10 900 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/self_launch_2.log 2>&1 || { tail -40 $O/self_launch_2.log; exit 1; }
grep '^{' $O/self_launch_2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['n_gpus'], d.get('dp_scatter'))"
