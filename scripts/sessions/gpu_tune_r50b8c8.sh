set -o pipefail
o=gpurun_out/r50c8; mkdir -p $o
PYTHONPATH=. timeout -k 10 300 python scripts/sweep_dyn.py --points 8,8,64,200 16,6,96,200 --iters 200 > $o/sweep_old.jsonl 2>&1 || exit 1
timeout -k 10 400 python -m hipzap.engine.tune --batch 8 16 --concurrent 8 6 --report $o/tune.json > $o/tune.log 2>&1 || exit 2
cp hipzap/tuning/resnet50_bs8_c8.json hipzap/tuning/resnet50_bs16_c6.json $o/ 2>/dev/null
PYTHONPATH=. timeout -k 10 300 python scripts/sweep_dyn.py --points 8,8,64,200 16,6,96,200 --iters 200 > $o/sweep_new.jsonl 2>&1 || exit 3
