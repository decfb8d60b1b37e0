#!/usr/bin/env bash
# End-to-end HTTP serving sweep of the three topologies on one MI355X (closed-loop users).
set -euo pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/load
timeout -k 10 ${SWEEP_TIMEOUT:-1000} python scripts/serving_sweep.py --archs ${ARCHS:-monolithic,triton,microservices} \
  --users ${USERS:-1,10,50,100} --warmup ${WARMUP:-5} --measure ${MEASURE:-15} --procs ${PROCS:-4} \
  --procs-per-gpu ${PPG:-4} \
  --out gpurun_out/load 2>&1 | tee gpurun_out/load/sweep.log
