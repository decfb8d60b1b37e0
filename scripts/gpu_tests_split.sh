#!/usr/bin/env bash
# Run the GPU pipeline tests alone, then the whole GPU suite (diagnostic).
set -uo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
python tools/build_ext.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 400 python -m pytest tests/test_pipeline_gpu.py -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_pipe.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_pipe.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu.log
exit $rc
