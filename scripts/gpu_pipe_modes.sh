#!/usr/bin/env bash
set -uo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for m in 2 1 0; do
  ARENA_COPY_MODE=$m timeout -k 10 300 python -m pytest tests/test_pipeline_gpu.py -m gpu -q -p no:cacheprovider > gpurun_out/pipe_mode$m.log 2>&1
  echo "mode $m rc=$?: $(tail -1 gpurun_out/pipe_mode$m.log)"
done
