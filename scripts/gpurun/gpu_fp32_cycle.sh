#!/usr/bin/env bash
# One fp32 iteration: kernel tests -> retune the fp32 tables -> engine profile -> e2e bench.
# usage: [NOTUNE=1] [TESTS_K=<pytest -k expr>] scripts/gpurun/gpu_fp32_cycle.sh TAG
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-cycle}
mkdir -p gpurun_out/$T
$S 300 gpurun_out/$T/tests.log python -u -m pytest tests/test_fp32_gpu.py -k "${TESTS_K:-fp32 or x3 or ir}" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
grep -q "passed" gpurun_out/$T/tests.log && ! grep -q "failed" gpurun_out/$T/tests.log || { echo "tests failed"; exit 1; }
if [ "${NOTUNE:-0}" = "0" ]; then
  $S 400 gpurun_out/$T/tune.log python -u tools/tune_programs.py --dtypes fp32 --out gpurun_out/$T/conv_tuning.json --base data/tuning/conv_tuning.json || exit 1
  export ARENA_TUNING_FILE=gpurun_out/$T/conv_tuning.json
fi
bash scripts/gpurun/gpu_prof_fp32.sh $T/prof || exit 1
$S 400 gpurun_out/$T/bench.log python -u bench.py || exit 1
tail -2 gpurun_out/$T/bench.log
