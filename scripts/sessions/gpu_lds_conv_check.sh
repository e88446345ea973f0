set -o pipefail
mkdir -p gpurun_out/lds1
timeout -k 10 300 python -u -m pytest tests/test_conv_lds_gpu.py tests/test_vision_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lds1/pytest.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --mode scatter --global-batch 32 --steps 100 --warmup 10 --cold-trials 0 > gpurun_out/lds1/scatter_old_table.log 2>&1 || exit 2
timeout -k 10 200 python bench.py --mode scatter --global-batch 32 --steps 100 --warmup 10 --cold-trials 0 --tuned scripts/empty_tuning.json > gpurun_out/lds1/scatter_heur.log 2>&1 || exit 3
cp hipzap/tuning/resnet50_bs32.json gpurun_out/lds1/resnet50_bs32_old.json
timeout -k 10 500 python -m hipzap.engine.tune --batch 32 --report gpurun_out/lds1/tune_bs32_report.json > gpurun_out/lds1/tune.log 2>&1 || exit 4
cp hipzap/tuning/resnet50_bs32.json gpurun_out/lds1/resnet50_bs32_new.json
timeout -k 10 200 python bench.py --mode scatter --global-batch 32 --steps 100 --warmup 10 --cold-trials 0 > gpurun_out/lds1/scatter_new_table.log 2>&1 || exit 5
