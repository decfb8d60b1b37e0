#!/usr/bin/env bash
# Model-server arm (3 servers + 3 native gateways): ensemble dynamic-batching delay sweep.
set -euo pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1 ARENA_NATIVE_HTTP=1 LOG_LEVEL=WARNING ARENA_DECODE_PROCS=4
for d in ${DELAYS:-500 2000}; do
  O=gpurun_out/triton_d$d
  mkdir -p $O
  ARENA_ENSEMBLE_QUEUE_DELAY_US=$d timeout -k 10 300 python scripts/serving_sweep.py --archs triton \
    --users ${USERS:-10,50,100} --procs 4 --procs-per-gpu 3 --out $O > $O/sweep.log 2>&1
  echo "ensemble delay $d us"; grep "users=" $O/sweep.log
done
