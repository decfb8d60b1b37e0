#!/usr/bin/env bash
# GPU validation run used with gpurun: tests, smoke, short bench, rocprof stats.
set -euo pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
python tools/build_ext.py > gpurun_out/build.log 2>&1
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -50 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps ${STEPS:-100} --warmup 10 > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
