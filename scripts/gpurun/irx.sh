#!/usr/bin/env bash
# fused fp32-accurate 14x14/7x7 IR kernel (csrc/kernels/ir_crop_f32.hip): fp64-pinned tests, standalone timing,
# engine kernel traces with and without it.  usage: scripts/gpurun/irx.sh TAG
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-irx}
mkdir -p gpurun_out/$T
$S 300 gpurun_out/$T/tests.log python -u -m pytest tests/test_fp32_gpu.py -x -q -k "ir_block_f32" --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" gpurun_out/$T/tests.log && ! grep -q "failed" gpurun_out/$T/tests.log || { echo "tests failed"; exit 1; }
ARENA_IRC_F32=1 $S 200 gpurun_out/$T/bench_irc.log python -u tools/bench_irc.py --small || exit 1
cat gpurun_out/$T/bench_irc.log
for m in 1 0; do
  ARENA_IRC_F32=$m $S 300 gpurun_out/$T/prof$m.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/p$m -o eng -- python3 tools/profile_engine.py --dtype fp32 --batches 12 || exit 1
  f=$(find gpurun_out/$T/p$m -name "eng_kernel_trace.csv" | head -1)
  ARENA_IRC_F32=$m python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/$T/ops$m.md > /dev/null 2>&1; tail -14 gpurun_out/$T/ops$m.md
  rm -f "$f"
done
