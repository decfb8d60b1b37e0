#!/usr/bin/env bash
# x3h halo kernel iteration: numerics, standalone timing against the 16x16x32 halo kernels.  usage: TAG
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-x3hi}
mkdir -p gpurun_out/$T
$S 300 gpurun_out/$T/tests.log python -u -m pytest tests/test_fp32_gpu.py -x -q -k "x3h or x3g" --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" gpurun_out/$T/tests.log && ! grep -q "failed" gpurun_out/$T/tests.log || { echo "tests failed"; tail -30 gpurun_out/$T/tests.log; exit 1; }
$S 300 gpurun_out/$T/bench.log python -u tools/bench_x3g.py --impls 131,132,133,134,135,136,101,102,103,108,109,110,117,120 --shapes head_3x3,head_144,head_80,c3_3x3_32,c3_3x3_64,c3_3x3_128,head_144_40,stem_16 || exit 1
cat gpurun_out/$T/bench.log
bash scripts/gpurun/pmc_x3g.sh $T/pmc 131,132,134,136 head_3x3 > gpurun_out/$T/pmc.log 2>&1 || { tail gpurun_out/$T/pmc.log; exit 99; }
cat gpurun_out/$T/pmc.log
