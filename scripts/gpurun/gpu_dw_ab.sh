#!/usr/bin/env bash
# fp32 depthwise A/B: kernel tests, then the serialised engine's per-op table with ARENA_DW_CX=1 (one output
# column per thread) and the default (two).
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
$S 300 gpurun_out/dw_tests.log python -u -m pytest tests/test_fp32_gpu.py tests/test_kernels_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" gpurun_out/dw_tests.log && ! grep -q "failed" gpurun_out/dw_tests.log || { echo "tests failed"; exit 1; }
for cx in 1 2; do
  mkdir -p gpurun_out/dw_cx$cx
  ARENA_DW_CX=$cx $S 300 gpurun_out/dw_cx$cx/run.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dw_cx$cx -o eng -- python3 tools/profile_engine.py --dtype fp32 --batches 12 || exit 1
  f=$(find gpurun_out/dw_cx$cx -name "eng_kernel_trace.csv" | head -1)
  python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/dw_cx$cx/ops.md > /dev/null 2>&1
  find gpurun_out/dw_cx$cx -name "*.csv" -delete
  grep -E "dwconv|device time" gpurun_out/dw_cx$cx/ops.md
done
