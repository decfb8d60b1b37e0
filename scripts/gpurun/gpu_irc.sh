#!/usr/bin/env bash
# fused fp32 14x14/7x7 IR kernel: kernel tests, fp32 parity, retuned table, engine profile, short bench
# usage: scripts/gpurun/gpu_irc.sh TAG
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-irc}
mkdir -p gpurun_out/$T
$S 300 gpurun_out/$T/tests.log python -u -m pytest tests/test_fp32_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" gpurun_out/$T/tests.log && ! grep -q "failed" gpurun_out/$T/tests.log || { echo "tests failed"; exit 1; }
$S 400 gpurun_out/$T/tune.log python tools/tune_programs.py --out gpurun_out/$T/conv_tuning.json --base data/tuning/conv_tuning.json --dtypes fp32 || exit 1
cp gpurun_out/$T/conv_tuning.json data/tuning/conv_tuning.json
$S 300 gpurun_out/$T/run.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T -o eng -- python3 tools/profile_engine.py --dtype fp32 --batches 12 || exit 1
f=$(find gpurun_out/$T -name "eng_kernel_trace.csv" | head -1)
python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/$T/ops.md > /dev/null 2>&1; tail -14 gpurun_out/$T/ops.md
rm -f "$f"
$S 300 gpurun_out/$T/bench.log python bench.py --steps 60 --warmup 10 --bs1-requests 30 || exit 1
