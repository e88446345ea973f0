set -o pipefail
o=gpurun_out/mx8w; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --mode scatter --model vit-b16-fp8 --global-batch 64 --steps 50 --warmup 5 --cold-trials 0 > $o/scatter_old.log 2>&1 || exit 2
timeout -k 10 200 python scripts/bench_models.py vit-b16-fp8 > $o/models_old.jsonl 2>&1 || exit 3
cp hipzap/tuning/vit-b16-fp8_bs64.json $o/old_bs64.json; cp hipzap/tuning/vit-b16-fp8_bs8.json $o/old_bs8.json
timeout -k 10 500 python -m hipzap.engine.tune --model vit-b16-fp8 --batch 64 8 --report $o/tune_report.json > $o/tune.log 2>&1 || exit 4
cp hipzap/tuning/vit-b16-fp8_bs64.json $o/new_bs64.json; cp hipzap/tuning/vit-b16-fp8_bs8.json $o/new_bs8.json
timeout -k 10 200 python bench.py --mode scatter --model vit-b16-fp8 --global-batch 64 --steps 50 --warmup 5 --cold-trials 0 > $o/scatter_new.log 2>&1 || exit 5
timeout -k 10 200 python scripts/bench_models.py vit-b16-fp8 > $o/models_new.jsonl 2>&1 || exit 6
