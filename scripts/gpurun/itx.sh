#!/usr/bin/env bash
# tiled x3 IR kernel (csrc/kernels/ir_tile_x3.hip): fp64-pinned tests (both paths), pipeline parity, engine kernel
# traces with and without it, bench.  usage: scripts/gpurun/itx.sh TAG
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-itx}
mkdir -p gpurun_out/$T
$S 400 gpurun_out/$T/tests.log python -u -m pytest tests/test_fp32_gpu.py -x -q -k "ir_block_f32 or fp32_pipeline or fuses" --timeout 200 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" gpurun_out/$T/tests.log && ! grep -q "failed" gpurun_out/$T/tests.log || { echo "tests failed"; tail -40 gpurun_out/$T/tests.log; exit 1; }
for m in 1 0; do
  ARENA_IR_X3T=$m $S 300 gpurun_out/$T/prof$m.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/p$m -o eng -- python3 tools/profile_engine.py --dtype fp32 --batches 12 || exit 1
  f=$(find gpurun_out/$T/p$m -name "eng_kernel_trace.csv" | head -1)
  ARENA_IR_X3T=$m python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/$T/ops$m.md > /dev/null 2>&1; grep "device time" gpurun_out/$T/ops$m.md
  rm -f "$f"
done
grep "ir_tile_x3\|ir_f32_kernel" gpurun_out/$T/ops1.md | cut -c1-150
grep "ir_f32_kernel" gpurun_out/$T/ops0.md | cut -c1-150
$S 300 gpurun_out/$T/bench.log python bench.py --steps 20 --warmup 5 --no-secondary-bf16 || exit 1
tail -1 gpurun_out/$T/bench.log | cut -c1-400
