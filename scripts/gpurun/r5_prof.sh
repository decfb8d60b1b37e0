#!/usr/bin/env bash
# Late kernel change (fp32 head pool staged in two K halves): its tests first, then the closing profiles
# (r5_final.sh prof: op tables at bs 32 / 1, JPEG stage, PMC per op with durations).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-r5final}
mkdir -p gpurun_out/$T
$S 600 gpurun_out/$T/pytest_headpool.log python -u -m pytest tests/test_fp32_gpu.py -k "head_pool or matches_reference" tests/test_kernels_gpu.py -k head_pool tests/test_pipeline_gpu.py -k head_pool tests/test_headline_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
grep -E "passed|failed|error" gpurun_out/$T/pytest_headpool.log | tail -2
grep -q " failed\| error" gpurun_out/$T/pytest_headpool.log && exit 1
bash scripts/gpurun/r5_final.sh prof $T
