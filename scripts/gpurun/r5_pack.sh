#!/bin/bash
# Bench with the JPEG coefficients packed into the slot's staging (one DMA per batch) against per-upload DMAs.
set -o pipefail
mkdir -p gpurun_out/r5copy
ARENA_JPEG_PACK_COEFS=1 timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_jpeg_native_gpu.py \
  tests/test_headline_gpu.py tests/test_pipeline_gpu.py > gpurun_out/r5copy/pack_tests.log 2>&1 || { echo "pack tests failed"; tail -20 gpurun_out/r5copy/pack_tests.log; exit 1; }
tail -1 gpurun_out/r5copy/pack_tests.log
for p in 1 0; do
  ARENA_JPEG_PACK_COEFS=$p timeout -k 10 300 python -u bench.py > gpurun_out/r5copy/bench_pack$p.log 2>&1 || { echo "bench pack$p failed"; tail -5 gpurun_out/r5copy/bench_pack$p.log; exit 1; }
  grep '^{' gpurun_out/r5copy/bench_pack$p.log | tail -1 > gpurun_out/r5copy/bench_pack$p.json
  python -c "import json;d=json.load(open('gpurun_out/r5copy/bench_pack$p.json'));print('pack $p', d['value'], d['engine_req_s'], d['engine_rgb_req_s'], d['bf16']['value'], d['p99_ms'], d['host_cpu_us_per_req']['total'])"
done
