set -o pipefail
o=gpurun_out/http_dyn; mkdir -p $o
timeout -k 10 200 python -u scripts/http_load.py --native --contexts 24 --clients 32 --requests 300 --format npy > $o/npy_b1.json 2> $o/npy_b1.err || exit 1
timeout -k 10 200 python -u scripts/http_load.py --native --contexts 8 --plan-batch 8 --clients 64 --requests 200 --format npy > $o/npy_b8.json 2> $o/npy_b8.err || exit 2
timeout -k 10 200 python -u scripts/http_load.py --native --contexts 8 --plan-batch 8 --clients 64 --requests 200 --format json > $o/json_b8.json 2> $o/json_b8.err || exit 3
timeout -k 10 200 python -u scripts/http_load.py --native --contexts 24 --clients 32 --requests 300 --format json > $o/json_b1.json 2> $o/json_b1.err || exit 4
