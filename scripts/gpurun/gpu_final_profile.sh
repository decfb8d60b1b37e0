#!/usr/bin/env bash
# Per-op fp32 kernel table of HEAD (rocprofv3 kernel trace of the serialised engine, mapped back to program
# ops), a bs=1 trace (graph node count + device time) and a counter pass over the fp32 engine.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
mkdir -p gpurun_out/prof_final gpurun_out/prof_bs1
$S 300 gpurun_out/prof_final/run.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final -o eng -- python3 tools/profile_engine.py --dtype fp32 --batches 12 || exit 1
f=$(find gpurun_out/prof_final -name "eng_kernel_trace.csv" | head -1)
python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/prof_final/ops.md > /dev/null 2>&1; tail -16 gpurun_out/prof_final/ops.md
$S 300 gpurun_out/prof_bs1/run.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bs1 -o bs1 -- python3 tools/profile_engine.py --dtype fp32 --batch 1 --batches 12 || exit 1
f=$(find gpurun_out/prof_bs1 -name "bs1_kernel_trace.csv" | head -1)
python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/prof_bs1/ops.md > /dev/null 2>&1; tail -16 gpurun_out/prof_bs1/ops.md
