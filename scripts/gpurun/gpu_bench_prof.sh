#!/usr/bin/env bash
# e2e bench (short) + rocprofv3 kernel trace of the engine-only fp32 path; outputs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
mkdir -p gpurun_out/prof_fp32
$S 400 gpurun_out/bench_e2e.log python bench.py --steps ${STEPS:-40} --warmup 10 --bs1-requests 30 ${BENCH_ARGS:-} || exit 1
grep '^{' gpurun_out/bench_e2e.log > gpurun_out/bench_e2e.json || true
$S 300 gpurun_out/prof_fp32/run.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fp32 -o eng -- python3 tools/profile_engine.py --dtype ${PDTYPE:-fp32} --batches 12 || exit 1
f=$(find gpurun_out/prof_fp32 -name "eng_kernel_trace.csv" | head -1)
[ -n "$f" ] && python tools/analyze_trace.py "$f" --dtype ${PDTYPE:-fp32} --replays 8 --out gpurun_out/prof_fp32/ops.md > /dev/null 2>&1; tail -12 gpurun_out/prof_fp32/ops.md
