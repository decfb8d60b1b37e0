#!/usr/bin/env bash
# fp32 iteration loop: fp32 numerics tests, engine kernel trace (per-op table), short HTTP bench.
# usage: scripts/gpurun/iter_fp32.sh TAG [pytest -k expr]
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-iter}
K=${2:-}
mkdir -p gpurun_out/$T
if [ -n "$K" ]; then
  $S 400 gpurun_out/$T/tests.log python -u -m pytest tests/test_fp32_gpu.py -x -q -k "$K" --timeout 200 --timeout-method thread -p no:cacheprovider || exit 1
else
  $S 400 gpurun_out/$T/tests.log python -u -m pytest tests/test_fp32_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider || exit 1
fi
grep -q " passed" gpurun_out/$T/tests.log && ! grep -q "failed" gpurun_out/$T/tests.log || { echo "tests failed"; tail -40 gpurun_out/$T/tests.log; exit 1; }
$S 300 gpurun_out/$T/prof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/p -o eng -- python3 tools/profile_engine.py --dtype fp32 --batches 12 || exit 1
f=$(find gpurun_out/$T/p -name "eng_kernel_trace.csv" | head -1)
python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/$T/ops.md > /dev/null 2>&1; grep "device time" gpurun_out/$T/ops.md
rm -f "$f"
$S 300 gpurun_out/$T/bench.log python bench.py --steps 20 --warmup 5 --no-secondary-bf16 --no-secondary-inproc --latency-levels '' || exit 1
tail -1 gpurun_out/$T/bench.log | cut -c1-300
