#!/usr/bin/env bash
# Does the head-lanes crash of the arm-B detection service come from its 2 hardware queues per process?
# The lanes bit-identity test with GPU_MAX_HW_QUEUES=4 (HIP's default) and =2 (start_arena's setting for 5 GPU
# processes per device); each in its own time-limited step.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4lanesq
for q in 4 2; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -k head_lanes -x -q --timeout 180 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r4lanesq/q$q.log 2>&1
  rc=$?
  echo "queues=$q rc=$rc $(grep -E 'passed|failed|Segmentation|Fatal' gpurun_out/r4lanesq/q$q.log | tail -1)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 0; fi  # a crash / abort / timeout: nothing more on the GPU
done
