#!/usr/bin/env bash
# Microservices arm (3 detection + 2 classification processes, queue cap on): classifier queue delay sweep.
set -euo pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1 ARENA_NATIVE_HTTP=1 LOG_LEVEL=WARNING ARENA_CROP_TRANSPORT=raw ARENA_FANOUT=batch
export ARENA_DECODE_PROCS=3 ARENA_CLS_PROCS_PER_GPU=2
for d in ${DELAYS:-500 2000 4000}; do
  O=gpurun_out/micro_clsd$d
  mkdir -p $O
  ARENA_CLS_QUEUE_DELAY_US=$d timeout -k 10 300 python scripts/serving_sweep.py --archs microservices \
    --users ${USERS:-10,50,100} --procs 4 --procs-per-gpu 3 --out $O > $O/sweep.log 2>&1
  echo "cls delay $d us"; grep "users=" $O/sweep.log
done
