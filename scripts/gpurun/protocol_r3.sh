#!/usr/bin/env bash
# Long-phase protocol runs: one arm, given user levels, 10 s warm-up + 60 s measurement,
# 3 runs per level (reference experiment.yaml:303-314 uses 60 s warm-up / 180 s / 30 s cooldown; shortened to fit
# the 20-minute call limit).  ENVELOPE=2 confines every service process to 2 CPUs of its own (ARENA_SERVICE_CPUS).
# usage: scripts/gpurun/protocol_r3.sh ARCH USERS TAG
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1 ARENA_NATIVE_HTTP=1 LOG_LEVEL=WARNING ARENA_CROP_TRANSPORT=raw ARENA_FANOUT=batch
ARCH=$1; U=$2; T=${3:-protocol_r3}
O=gpurun_out/$T/$ARCH
mkdir -p $O
export ARENA_SERVICE_CPUS=${ENVELOPE:-0}
case $ARCH in
  monolithic) export ARENA_DECODE_PROCS=${DECODE:-8}; PPG=1 ;;
  triton) export ARENA_DECODE_PROCS=${DECODE:-4}; PPG=3 ;;
  microservices) export ARENA_DECODE_PROCS=${DECODE:-3} ARENA_CLS_PROCS_PER_GPU=2; PPG=3 ;;
esac
[ "${ENVELOPE:-0}" != "0" ] && PPG=1
timeout -k 10 1100 python scripts/serving_sweep.py --archs $ARCH --users $U --procs 4 --procs-per-gpu $PPG \
  --warmup 10 --measure 60 --cooldown 2 --runs 3 --out $O > $O/sweep.log 2>&1
# keep what the analysis reads (summaries, CSV, hypotheses, the sweep log); server logs can exceed gpurun's
# 64 MiB copy-back limit
find $O -type f -size +2M -delete
grep -h "users=" $O/sweep.log
