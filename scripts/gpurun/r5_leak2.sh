#!/bin/bash
# Memory growth A/B on the device-JPEG serving path: per-JPEG DMAs from pooled buffers vs coefficients packed into
# the slot's staging (ARENA_JPEG_PACK_COEFS=1), plus the JPEG GPU tests with packing on.
set -o pipefail
mkdir -p gpurun_out/r5leak
export ARENA_JPEG_PACK_COEFS=1
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_jpeg_native_gpu.py \
  > gpurun_out/r5leak/pack_tests.log 2>&1 || { echo "pack tests rc=$?"; tail -20 gpurun_out/r5leak/pack_tests.log; exit 1; }
tail -2 gpurun_out/r5leak/pack_tests.log
timeout -k 10 200 python -u tools/leak_probe.py --gpu --rounds 6 --per-round 30000 > gpurun_out/r5leak/srv3_pack.log 2>&1
echo "== pack rc=$?"; cat gpurun_out/r5leak/srv3_pack.log | grep round
unset ARENA_JPEG_PACK_COEFS
timeout -k 10 200 python -u tools/leak_probe.py --gpu --rounds 6 --per-round 30000 > gpurun_out/r5leak/srv3_dma.log 2>&1
echo "== dma rc=$?"; cat gpurun_out/r5leak/srv3_dma.log | grep round
