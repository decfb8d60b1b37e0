#!/usr/bin/env bash
# Model-server arm (3 servers + 3 gateways on one GPU): HIP's default 4 hardware queues per process vs 2.
set -euo pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1 ARENA_NATIVE_HTTP=1 LOG_LEVEL=WARNING ARENA_DECODE_PROCS=4
for q in 4 2; do
  O=gpurun_out/triton_hwq_$q
  mkdir -p $O
  ARENA_HW_QUEUES=$q timeout -k 10 400 python scripts/serving_sweep.py --archs triton --users ${USERS:-1,10,100} \
    --procs 4 --procs-per-gpu 3 --out $O > $O/sweep.log 2>&1
  grep "users=" $O/sweep.log
done
