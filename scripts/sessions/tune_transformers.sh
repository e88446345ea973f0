set -e
mkdir -p gpurun_out/tune2
timeout -k 10 300 python -u -m hipzap.engine.tune --model bert-base --batch 16 --report gpurun_out/tune2/tune_bert.json > gpurun_out/tune2/tune_bert.log 2>&1
timeout -k 10 300 python -u -m hipzap.engine.tune --model vit-b16 --batch 8 --report gpurun_out/tune2/tune_vit.json > gpurun_out/tune2/tune_vit.log 2>&1
timeout -k 10 300 python -u -m hipzap.engine.tune --model vit-b16-fp8 --batch 8 64 --report gpurun_out/tune2/tune_vit8.json > gpurun_out/tune2/tune_vit8.log 2>&1
cp hipzap/tuning/bert-base_bs16.json hipzap/tuning/vit-b16_bs8.json hipzap/tuning/vit-b16-fp8_bs8.json hipzap/tuning/vit-b16-fp8_bs64.json gpurun_out/tune2/
timeout -k 10 300 python -u scripts/bench_models.py > gpurun_out/tune2/bench_models.jsonl 2> gpurun_out/tune2/bench_models.err
