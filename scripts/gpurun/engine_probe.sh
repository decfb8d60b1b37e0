#!/usr/bin/env bash
# Engine-only throughput under staging / concurrency knobs, and a bs=1 fp32 kernel trace.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-probe}
mkdir -p gpurun_out/$T
$S 200 gpurun_out/$T/e0.log python tools/engine_probe.py || exit 1
grep engine gpurun_out/$T/e0.log
ARENA_DEBUG_SKIP_PACK=12 $S 200 gpurun_out/$T/e1.log python tools/engine_probe.py || exit 1
grep engine gpurun_out/$T/e1.log
ARENA_SLOTS=6 ARENA_CONCURRENCY=4 $S 200 gpurun_out/$T/e2.log python tools/engine_probe.py || exit 1
grep engine gpurun_out/$T/e2.log
$S 300 gpurun_out/$T/prof1.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/p1 -o eng -- python3 tools/profile_engine.py --dtype fp32 --batch 1 --batches 30 || exit 1
f=$(find gpurun_out/$T/p1 -name "eng_kernel_trace.csv" | head -1)
python tools/analyze_trace.py "$f" --dtype fp32 --replays 20 --out gpurun_out/$T/ops_bs1.md > /dev/null 2>&1; grep "device time" gpurun_out/$T/ops_bs1.md
rm -f "$f"
