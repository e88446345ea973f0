# HIP runtime init cost under environment variants (fresh process each trial, interleaved)
o=gpurun_out/initenv; mkdir -p $o
for t in 1 2 3 4 5 6 7; do
  for v in base HSA_ENABLE_INTERRUPT=0 HSA_ENABLE_SDMA=0 AMD_LOG_LEVEL=0 HIP_FORCE_DEV_KERNARG=1 HSA_ENABLE_SCRATCH_ASYNC_RECLAIM=0 GPU_MAX_HW_QUEUES=1; do
    if [ $v = base ]; then timeout -k 5 30 ./scripts/native/hip_init_probe > $o/tmp.json 2>/dev/null || exit 1
    else env $v timeout -k 5 30 ./scripts/native/hip_init_probe > $o/tmp.json 2>/dev/null || exit 1; fi
    echo "{\"env\": \"$v\", \"r\": $(cat $o/tmp.json)}" >> $o/sweep.jsonl
  done
done
