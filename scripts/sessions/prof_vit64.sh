set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
o=gpurun_out/vit64; mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o vit -- python3 bench.py --mode scatter --model vit-b16-fp8 --global-batch 64 --steps 20 --warmup 3 --cold-trials 0 > $o/bench.log 2>&1 || exit 1
