#!/usr/bin/env bash
# tests + smoke + bench + rocprof profile in one gpurun call (stops at the first failure)
set -euo pipefail
cd "$(dirname "$0")/../.."
bash scripts/gpurun/gpu_check.sh
STEPS=${PSTEPS:-30} bash scripts/gpurun/gpu_profile.sh > /dev/null
python tools/analyze_trace.py gpurun_out/prof/bench_kernel_trace.csv --out gpurun_out/prof/ops.md | tail -14
