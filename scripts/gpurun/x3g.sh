#!/usr/bin/env bash
# x3g kernels (csrc/kernels/gemm_x3.hip): fp64-pinned tests, then the per-layer sweep of every fp32 conv of the
# pipeline against the existing kernels.  usage: scripts/gpurun/x3g.sh TAG
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-x3g}
mkdir -p gpurun_out/$T
$S 300 gpurun_out/$T/tests.log python -u -m pytest tests/test_fp32_gpu.py -x -q -k "x3g or conv_f32_matches" --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" gpurun_out/$T/tests.log && ! grep -q "failed" gpurun_out/$T/tests.log || { echo "tests failed"; exit 1; }
$S 400 gpurun_out/$T/sweep.log python -u tools/bench_f32_convs.py --iters 20 --variants 0,1,2,3,4,5,7,9,10,12,13,14 --x3 0,1,4,5,6,7,8 --out gpurun_out/$T/variants.md || exit 1
tail -5 gpurun_out/$T/variants.md
