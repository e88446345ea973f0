#!/bin/bash
# r5 s29: register-staged MX-fp8 tile (cfg 51: two k-steps in flight at cfg 24's LDS / residency):
# bitwise vs cfg 24, oracle tests, ViT bs64 microbench against cfg 24; then the L2 / wait PMC passes
# of cfg 24, cfg 51 and hipBLASLt's fp8 kernel on the same shapes
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s29; mkdir -p $O
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_fp8_gpu.py -k "mx8_activations or mx256" > $O/pytest.log 2>&1
echo "pytest rc=$?"
grep -E 'FAILED|ERROR|passed|failed' $O/pytest.log | tail -12
timeout -k 10 300 python3 scripts/bench_mx.py --cfgs 24,51 > $O/mx.jsonl 2> $O/mx.err || { tail -5 $O/mx.err; exit 1; }
python3 -c "
import json
for l in open('$O/mx.jsonl'):
    if l.startswith('{'):
        j = json.loads(l); print(j['shape'], j['best_cfg'], {c: v['us'] for c, v in j['cfgs'].items()})"
fi
T="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES"
S="SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES"
for c in 24 51; do
  timeout -s KILL 90 rocprofv3 --pmc $T -d $O/c${c}_T -o p --output-format csv -- python3 scripts/bench_mx.py --cfgs $c > $O/c${c}_T.log 2>&1 || { echo "c${c}_T failed"; tail -5 $O/c${c}_T.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc $S -d $O/c${c}_S -o p --output-format csv -- python3 scripts/bench_mx.py --cfgs $c > $O/c${c}_S.log 2>&1 || { echo "c${c}_S failed"; tail -5 $O/c${c}_S.log; exit 1; }
done
timeout -s KILL 90 rocprofv3 --pmc $T -d $O/lib_T -o p --output-format csv -- python3 scripts/bench_mx.py --torch > $O/lib_T.log 2>&1 || { echo "lib_T failed"; tail -5 $O/lib_T.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc $S -d $O/lib_S -o p --output-format csv -- python3 scripts/bench_mx.py --torch > $O/lib_S.log 2>&1 || { echo "lib_S failed"; tail -5 $O/lib_S.log; exit 1; }
du -sh $O/*_T $O/*_S
python3 scripts/pmc_summary.py $O/c24_T $O/c24_S $O/c51_T $O/c51_S $O/lib_T $O/lib_S $O/pmc.json
rm -rf $O/c24_T $O/c24_S $O/c51_T $O/c51_S $O/lib_T $O/lib_S
python3 - <<PY
import json
d = json.load(open("$O/pmc.json"))
for run, v in d.items():
    for k, c in v["per_kernel"].items():
        if c.get("dispatches", 0) < 20 or "elementwise" in k or "copy" in k: continue
        print(run, k[:60], c["dispatches"], {n: round(x / c["dispatches"]) for n, x in c.items() if n != "dispatches"})
PY
