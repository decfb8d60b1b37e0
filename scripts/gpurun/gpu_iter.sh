#!/usr/bin/env bash
# Quick iteration: selected GPU tests (PYTEST_K), then bench, then a kernel-trace profile.
set -euo pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
python tools/build_ext.py > gpurun_out/build.log 2>&1
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x ${PYTEST_K:+-k "$PYTEST_K"} \
  > gpurun_out/pytest_iter.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_iter.log; exit 1; }
tail -3 gpurun_out/pytest_iter.log
timeout -k 10 300 python bench.py --steps ${STEPS:-100} --warmup 10 > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
if [ "${PROFILE:-1}" = "1" ]; then
  STEPS=30 bash scripts/gpurun/gpu_profile.sh > /dev/null
  python tools/analyze_trace.py gpurun_out/prof/bench_kernel_trace.csv --out gpurun_out/prof/ops.md | tail -16
fi
