#!/usr/bin/env bash
# Microservices-arm serving sweeps on one MI355X with the native handler front end (server/native_handler.py),
# over the number of classification processes per GPU.
set -euo pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1 ARENA_NATIVE_HTTP=1 ARENA_CROP_TRANSPORT=raw ARENA_FANOUT=batch LOG_LEVEL=WARNING
export ARENA_DECODE_PROCS=${ARENA_DECODE_PROCS:-4} ARENA_QUEUE_DELAY_US=${ARENA_QUEUE_DELAY_US:-2000}
for k in ${CLS_PROCS:-1 2}; do
  mkdir -p gpurun_out/micro_cls$k
  ARENA_CLS_PROCS_PER_GPU=$k timeout -k 10 ${SWEEP_TIMEOUT:-420} python scripts/serving_sweep.py --archs microservices \
    --users ${USERS:-50,100,200} --warmup 5 --measure ${MEASURE:-15} --procs 4 --procs-per-gpu ${PPG:-2} \
    --out gpurun_out/micro_cls$k > gpurun_out/micro_cls$k/sweep.log 2>&1
  grep "users=" gpurun_out/micro_cls$k/sweep.log
done
