set -u
mkdir -p gpurun_out/r3_rpack
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_pth_lite_gpu.py tests/test_lmbatch_gpu.py > gpurun_out/r3_rpack/pytest.log 2>&1 || { tail -30 gpurun_out/r3_rpack/pytest.log; exit 1; }
tail -2 gpurun_out/r3_rpack/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_rpack/smoke.log 2>&1 || { tail -20 gpurun_out/r3_rpack/smoke.log; exit 1; }
tail -1 gpurun_out/r3_rpack/smoke.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3_rpack/bench_n1.log 2>&1 || { tail -20 gpurun_out/r3_rpack/bench_n1.log; exit 1; }
grep "^{" gpurun_out/r3_rpack/bench_n1.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.readline())
print(d['value'], d['cold_start_ms_p50'], d['cold_start_pth_torch_ms_p50'], d['cold_start_inprocess_ms_first'], d['cold_start_inprocess_breakdown_ms'])
print(d['cold_start_fresh_process']['pth']['median_trial_phases_ms'])"
