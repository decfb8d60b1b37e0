#!/usr/bin/env bash
# x3hg iteration: kernel numerics tests, then standalone timings of the 3x3 s1 layers vs the halo kernels.
# usage: scripts/gpurun/x3hg_iter.sh TAG
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-x3hg}
mkdir -p gpurun_out/$T
$S 300 gpurun_out/$T/tests.log python -u -m pytest tests/test_fp32_gpu.py -x -q -k "x3hg" --timeout 200 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" gpurun_out/$T/tests.log && ! grep -q "failed" gpurun_out/$T/tests.log || { echo "tests failed"; tail -40 gpurun_out/$T/tests.log; exit 1; }
$S 300 gpurun_out/$T/bench.log python -u tools/bench_x3g.py --iters 30 \
  --shapes ${SHAPES:-head_144,head_3x3,head_80,head_144_40,c3_3x3_64,c3_3x3_32,c3_3x3_128} \
  --impls ${IMPLS:-101,102,108,109,$(seq -s, 131 144)} || exit 1
cat gpurun_out/$T/bench.log
