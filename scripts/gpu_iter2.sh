#!/usr/bin/env bash
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x -k "conv or pipeline or ir_block or pointwise" > gpurun_out/pytest_iter.log 2>&1 || { tail -60 gpurun_out/pytest_iter.log; exit 1; }
tail -1 gpurun_out/pytest_iter.log
for v3 in 1 0; do
  ARENA_CONV_V3=$v3 timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/bench_v3_$v3.json 2> gpurun_out/bench_v3_$v3.err
  python -c "import json;d=json.load(open('gpurun_out/bench_v3_$v3.json'));print('v3=$v3', d['value'], d['p50_ms'], d['bs1_p50_ms'])"
done
timeout -k 10 300 python tools/bench_convs.py --impls 2,3 --iters 30 --out gpurun_out/convs.md > /dev/null
STEPS=30 bash scripts/gpu_profile.sh > /dev/null
python tools/analyze_trace.py gpurun_out/prof/bench_kernel_trace.csv --out gpurun_out/prof/ops.md | tail -14
