#!/bin/bash
# HIP runtime knobs against the resident set of tools/microbench/rss_hip (one run each).
mkdir -p gpurun_out
o=gpurun_out/r5_rss_hip_env.txt
: > $o
for e in "X=1" "HIP_INITIAL_DM_SIZE=0" "GPU_PINNED_XFER_SIZE=4" "GPU_STAGING_BUFFER_SIZE=1" "GPU_XFER_BUFFER_SIZE=1" "HSA_KERNARG_POOL_SIZE=1048576" "ROC_AQL_QUEUE_SIZE=1024" "GPU_MAX_HW_QUEUES=1" "ROC_SIGNAL_POOL_SIZE=64" "GPU_RESOURCE_CACHE_SIZE=0"; do
  echo "== $e" >> $o
  env $e timeout -k 5 30 ./tools/microbench/rss_hip >> $o 2>&1 || { echo "rc $?" >> $o; break; }
done
