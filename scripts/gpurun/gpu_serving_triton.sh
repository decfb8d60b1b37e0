#!/usr/bin/env bash
# Model-server ("triton") arm serving sweeps on one MI355X: native handler gateway (server/native_handler.py),
# spawned decode processes in the model server, over the number of model-server / gateway processes.
set -euo pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1 ARENA_NATIVE_HTTP=1 LOG_LEVEL=WARNING
export ARENA_DECODE_PROCS=${ARENA_DECODE_PROCS:-4}
for k in ${PPGS:-2 3}; do
  mkdir -p gpurun_out/triton_ppg$k
  timeout -k 10 ${SWEEP_TIMEOUT:-420} python scripts/serving_sweep.py --archs triton \
    --users ${USERS:-50,100,200} --warmup 5 --measure ${MEASURE:-15} --procs 4 --procs-per-gpu $k \
    --out gpurun_out/triton_ppg$k > gpurun_out/triton_ppg$k/sweep.log 2>&1
  grep "users=" gpurun_out/triton_ppg$k/sweep.log
done
