set -o pipefail
O=gpurun_out/dyn1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dyn_batch_gpu.py tests/test_conv_lds_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || exit 2
timeout -k 10 200 python bench.py --cold-trials 0 --cold-runs 0 --dyn-batch 16 --dyn-contexts 4 --dyn-clients 64 > $O/bench_dyn16.log 2>&1 || exit 3
