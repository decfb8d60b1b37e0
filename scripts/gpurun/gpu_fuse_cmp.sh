#!/usr/bin/env bash
# IR kernel tests, then bench under each fusion policy, then profile the default.
set -euo pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x -k "ir_block or pipeline" > gpurun_out/pytest_iter.log 2>&1 || { tail -60 gpurun_out/pytest_iter.log; exit 1; }
tail -1 gpurun_out/pytest_iter.log
for pol in all auto none; do
  ARENA_FUSE_IR=$pol timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/bench_$pol.json 2> gpurun_out/bench_$pol.err
  python -c "import json;d=json.load(open('gpurun_out/bench_$pol.json'));print('$pol', d['value'], d['p50_ms'], d['bs1_p50_ms'])"
done
STEPS=30 bash scripts/gpurun/gpu_profile.sh > /dev/null
python tools/analyze_trace.py gpurun_out/prof/bench_kernel_trace.csv --out gpurun_out/prof/ops.md | tail -16
