#!/bin/bash
# r5 s12: AWD-LSTM split first layer (W_hh0 h0 pre-pass in the layer-1 launch + cell0 launch):
# bitwise tests, then an interleaved A/B of HIPZAP_LM_SPLIT=0/1 (lone request, 32 / 64 clients),
# and a kernel trace of the split engine at 1 and 32 clients
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5_s12; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 180 --timeout-method thread -m gpu tests/test_lmbatch_gpu.py tests/test_lmlite_gpu.py > $O/pytest.log 2>&1
echo "pytest rc=$?"
grep -E 'FAILED|ERROR|passed|failed' $O/pytest.log | tail -25
for rep in 1 2; do
  for sp in 0 1; do
    HIPZAP_LM_SPLIT=$sp timeout -k 10 300 python3 scripts/bench_lm_batch.py --clients 1 32 64 --requests 12 > $O/lm_split${sp}_$rep.json 2> $O/lm_split${sp}_$rep.err || { tail -20 $O/lm_split${sp}_$rep.err; exit 1; }
    python3 -c "
import json; j=json.loads(open('$O/lm_split${sp}_$rep.json').read().strip().splitlines()[-1])
print('split=$sp rep $rep single', j['single_request_ms'], j['single_us_per_step'], [(l['clients'], l['req_per_s'], l['us_per_step'], l['p50_ms']) for l in j['load']])"
  done
done
for c in 1 32; do
  HIPZAP_LM_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p$c -o run -- python3 scripts/bench_lm_batch.py --clients $c --requests 4 > $O/prof_c$c.log 2>&1 || { tail -20 $O/prof_c$c.log; exit 1; }
  db=$(find $O/p$c -name '*results.db' | head -1)
  python3 scripts/rocpd_stats.py "$db" 20 > $O/kernel_stats_c$c.txt
  python3 scripts/rocpd_stats.py "$db" --timeline lmb_cell0 lmb_dec_kernel > $O/one_step_c$c.txt
  rm -rf $O/p$c
  cut -c1-150 $O/kernel_stats_c$c.txt | head -12; cat $O/one_step_c$c.txt
done
