#!/usr/bin/env bash
# conv kernel tests for every impl + per-layer microbenchmark
set -euo pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider -x -k "conv" > gpurun_out/pytest_conv.log 2>&1 || { tail -60 gpurun_out/pytest_conv.log; exit 1; }
tail -1 gpurun_out/pytest_conv.log
timeout -k 10 600 python tools/bench_convs.py --impls ${IMPLS:-2,3} --out gpurun_out/convs.md
