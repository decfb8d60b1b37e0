#!/usr/bin/env bash
# Closed-loop protocol runs of one arm (reference experiment.yaml:178-181,300-318) with the phases given in the
# environment: WARMUP / MEASURE / COOLDOWN seconds and RUNS per level (the reference: 60 / 180 / 30, 3 runs).
# Arm B's crop transport and fan-out come from TRANSPORT (jpeg = the reference's PIL JPEG q95 crops, raw, device)
# and FANOUT (parallel = one Classify RPC per crop under asyncio.gather, as the reference; batch = one
# ClassifyBatch); every level's summary JSON records the ARENA_* environment it ran with.
# ENVELOPE=2 confines every service process to 2 CPUs of its own (the reference's 2 vCPU containers).
# usage: scripts/gpurun/protocol.sh ARCH USERS TAG
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
ARCH=$1; U=$2; T=${3:-protocol}
export TMPDIR=/tmp PYTHONUNBUFFERED=1 ARENA_NATIVE_HTTP=1 LOG_LEVEL=WARNING
export ARENA_CROP_TRANSPORT=${TRANSPORT:-jpeg} ARENA_FANOUT=${FANOUT:-parallel}
W=${WARMUP:-10}; M=${MEASURE:-60}; C=${COOLDOWN:-2}; R=${RUNS:-3}
O=gpurun_out/$T/$ARCH${TAGSFX:-}
mkdir -p $O
export ARENA_SERVICE_CPUS=${ENVELOPE:-0}
case $ARCH in
  monolithic) export ARENA_DECODE_THREADS=${DTHREADS:-8} ARENA_DECODE_PROCS=2; PPG=1 ;;
  # one model-server process per GPU with batch overlap (round 5: 6.78k req/s at P99 19 ms and 4.9 model-server
  # CPUs at 100 users, 2.66k at 10 users; three processes: 6.93k at P99 22.6 ms, 7.0 CPUs, 1.98k at 10 users —
  # profiles/r5_serving/README.md)
  triton) export ARENA_DECODE_PROCS=${DECODE:-4}; PPG=1 ;;
  microservices) export ARENA_DECODE_PROCS=${DECODE:-3} ARENA_CLS_PROCS_PER_GPU=2; PPG=3 ;;
esac
if [ "${ENVELOPE:-0}" != "0" ]; then
  PPG=1
  export ARENA_DECODE_THREADS=${DTHREADS:-2}
fi
PPG=${PROCS_PER_GPU:-$PPG}  # serving processes per GPU (triton: model-server and gateway processes each)
LIMIT=$(( (W + M + C) * R * $(echo $U | tr ',' '\n' | wc -l) + 240 ))
timeout -k 10 $LIMIT python scripts/serving_sweep.py --archs $ARCH --users $U --procs 4 --procs-per-gpu $PPG \
  --warmup $W --measure $M --cooldown $C --runs $R --out $O > $O/sweep.log 2>&1
# keep what the analysis reads (summaries, CSV, hypotheses, the sweep log); server logs can exceed gpurun's
# 64 MiB copy-back limit: keep their last 256 KiB (a failed start's traceback is at the end)
for f in $(find $O -type f -size +2M); do tail -c 262144 "$f" > "$f.tail" && mv "$f.tail" "$f"; done
grep -h "users=" $O/sweep.log
