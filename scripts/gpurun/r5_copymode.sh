#!/bin/bash
# Input-DMA stream placement A/B: bench under ARENA_COPY_MODE 0 (shared copy stream), 2 (slot stream) and 3 (per-slot
# copy stream), then the device-JPEG memory probe under mode 3.
set -o pipefail
mkdir -p gpurun_out/r5copy
for m in 0 2 3; do
  ARENA_COPY_MODE=$m timeout -k 10 300 python -u bench.py > gpurun_out/r5copy/bench_m$m.log 2>&1 || { echo "bench m$m failed"; tail -5 gpurun_out/r5copy/bench_m$m.log; exit 1; }
  grep '^{' gpurun_out/r5copy/bench_m$m.log | tail -1 > gpurun_out/r5copy/bench_m$m.json
  python -c "import json;d=json.load(open('gpurun_out/r5copy/bench_m$m.json'));print('mode $m', d['value'], d['engine_req_s'], d['engine_rgb_req_s'], d['bf16']['value'], d['p99_ms'])"
done
ARENA_COPY_MODE=3 timeout -k 10 200 python -u tools/leak_probe.py --gpu --rounds 6 --per-round 30000 > gpurun_out/r5copy/srv_m3.log 2>&1
echo "== m3 rc=$?"; grep round gpurun_out/r5copy/srv_m3.log
