#!/usr/bin/env bash
# one x3g iteration: numerics, standalone timing, counters.  usage: scripts/gpurun/x3g_iter.sh TAG IMPLS
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-x3gi}
IMPLS=${2:-111,112,113,114,115,116,117,118,119,120,121,122,123,124,125,126,127,128,129,130}
mkdir -p gpurun_out/$T
$S 300 gpurun_out/$T/tests.log python -u -m pytest tests/test_fp32_gpu.py -x -q -k "x3g" --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" gpurun_out/$T/tests.log && ! grep -q "failed" gpurun_out/$T/tests.log || { echo "tests failed"; exit 1; }
$S 300 gpurun_out/$T/bench.log python -u tools/bench_x3g.py --impls $IMPLS,21,40 || exit 1
cat gpurun_out/$T/bench.log
bash scripts/gpurun/pmc_x3g.sh $T/pmc 112,117,122,127 det_s2_64 > gpurun_out/$T/pmc.log 2>&1 || { tail gpurun_out/$T/pmc.log; exit 99; }
cat gpurun_out/$T/pmc.log
