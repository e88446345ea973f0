set -o pipefail
o=gpurun_out/mx4s; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --mode scatter --model vit-b16-fp8 --global-batch 64 --steps 50 --warmup 5 --cold-trials 0 > $o/scatter_old.log 2>&1 || exit 2
timeout -k 10 300 python scripts/bench_models.py vit-b16-fp8 bert-base-fp8 > $o/models_old.jsonl 2>&1 || exit 3
timeout -k 10 500 python -m hipzap.engine.tune --model vit-b16-fp8 --batch 64 8 --report $o/tune_vit.json > $o/tune_vit.log 2>&1 || exit 4
timeout -k 10 300 python -m hipzap.engine.tune --model bert-base-fp8 --batch 16 --report $o/tune_bert.json > $o/tune_bert.log 2>&1 || exit 5
cp hipzap/tuning/vit-b16-fp8_bs64.json hipzap/tuning/vit-b16-fp8_bs8.json hipzap/tuning/bert-base-fp8_bs16.json $o/
timeout -k 10 200 python bench.py --mode scatter --model vit-b16-fp8 --global-batch 64 --steps 50 --warmup 5 --cold-trials 0 > $o/scatter_new.log 2>&1 || exit 6
timeout -k 10 300 python scripts/bench_models.py vit-b16-fp8 bert-base-fp8 > $o/models_new.jsonl 2>&1 || exit 7
