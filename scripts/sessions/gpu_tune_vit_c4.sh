set -o pipefail
o=gpurun_out/vitc4; mkdir -p $o
timeout -k 10 300 python scripts/bench_models.py vit-b16 > $o/models_old.jsonl 2>&1 || exit 1
timeout -k 10 400 python -m hipzap.engine.tune --model vit-b16 --batch 8 --concurrent 4 --report $o/tune.json > $o/tune.log 2>&1 || exit 2
cp hipzap/tuning/vit-b16_bs8_c4.json $o/
timeout -k 10 300 python scripts/bench_models.py vit-b16 > $o/models_new.jsonl 2>&1 || exit 3
