#!/bin/bash
# Memory growth on the device-JPEG serving path with one pinned allocation per pooled buffer (no carving).
set -o pipefail
mkdir -p gpurun_out/r5leak
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_jpeg_native_gpu.py tests/test_headline_gpu.py \
  > gpurun_out/r5leak/pool_tests.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/r5leak/pool_tests.log; exit 1; }
tail -2 gpurun_out/r5leak/pool_tests.log
timeout -k 10 240 python -u tools/leak_probe.py --gpu --rounds 8 --per-round 30000 > gpurun_out/r5leak/srv4_pool.log 2>&1
echo "== pool rc=$?"; grep round gpurun_out/r5leak/srv4_pool.log
