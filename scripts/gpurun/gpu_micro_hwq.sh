#!/usr/bin/env bash
# Microservices arm (3 detection + 2 classification processes on one GPU): default hardware queues per
# process vs GPU_MAX_HW_QUEUES=2 (five processes x 4 queues may oversubscribe the GPU's hardware queues).
set -euo pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1 ARENA_NATIVE_HTTP=1 LOG_LEVEL=WARNING ARENA_CROP_TRANSPORT=raw ARENA_FANOUT=batch
export ARENA_DECODE_PROCS=3 ARENA_CLS_PROCS_PER_GPU=2
for q in default 2; do
  O=gpurun_out/micro_hwq_$q
  mkdir -p $O
  if [ $q = default ]; then
    ARENA_HW_QUEUES=4 timeout -k 10 400 python scripts/serving_sweep.py --archs microservices --users ${USERS:-1,10,100} --procs 4 \
      --procs-per-gpu 3 --out $O > $O/sweep.log 2>&1
  else
    ARENA_HW_QUEUES=$q timeout -k 10 400 python scripts/serving_sweep.py --archs microservices --users ${USERS:-1,10,100} \
      --procs 4 --procs-per-gpu 3 --out $O > $O/sweep.log 2>&1
  fi
  grep "users=" $O/sweep.log
done
