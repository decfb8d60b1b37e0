#!/bin/bash
# Device-JPEG serving path memory on HEAD defaults (coefficients packed into the batch DMA), 8 rounds x 30k requests.
set -o pipefail
mkdir -p gpurun_out/r5leak
timeout -k 10 240 python -u tools/leak_probe.py --gpu --rounds 8 --per-round 30000 > gpurun_out/r5leak/srv6_head.log 2>&1
echo "== head rc=$?"; grep round gpurun_out/r5leak/srv6_head.log
