#!/bin/bash
# Memory growth on the device-JPEG serving path: per-JPEG DMAs on the compute stream (ARENA_COPY_MODE=2) and with
# batch overlap off, against the default (srv3_dma.log).
set -o pipefail
mkdir -p gpurun_out/r5leak
ARENA_COPY_MODE=2 timeout -k 10 200 python -u tools/leak_probe.py --gpu --rounds 6 --per-round 30000 > gpurun_out/r5leak/srv5_copymode2.log 2>&1
echo "== copymode2 rc=$?"; grep round gpurun_out/r5leak/srv5_copymode2.log
ARENA_BATCH_OVERLAP=0 timeout -k 10 200 python -u tools/leak_probe.py --gpu --rounds 6 --per-round 30000 > gpurun_out/r5leak/srv5_nooverlap.log 2>&1
echo "== nooverlap rc=$?"; grep round gpurun_out/r5leak/srv5_nooverlap.log
