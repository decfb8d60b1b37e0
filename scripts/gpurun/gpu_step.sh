#!/usr/bin/env bash
# Run one GPU step under its own time limit; stop the calling script on a fault / abort / timeout.
# usage: scripts/gpurun/gpu_step.sh SECONDS LOGFILE cmd...   (exit 0/1 = finished; anything else = stop)
set -u
secs=$1; log=$2; shift 2
mkdir -p "$(dirname "$log")"
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc: $*" >> "$log"
tail -3 "$log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
  echo "[gpu_step] stopping: rc=$rc ($*)"
  exit 99
fi
exit 0
