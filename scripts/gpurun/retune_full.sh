#!/usr/bin/env bash
# Retune the fp32 programs (base: the committed table), then the whole GPU tier, smoke, an fp32 engine kernel
# trace and the driver-shaped bench, all with the new table.  usage: scripts/gpurun/retune_full.sh TAG
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-retune}
mkdir -p gpurun_out/$T
$S 600 gpurun_out/$T/tune.log python tools/tune_programs.py --dtypes fp32 --base data/tuning/conv_tuning.json --out gpurun_out/$T/conv_tuning.json || exit 1
cp gpurun_out/$T/conv_tuning.json data/tuning/conv_tuning.json
$S 1000 gpurun_out/$T/pytest.log python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider || exit 1
tail -4 gpurun_out/$T/pytest.log
$S 300 gpurun_out/$T/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
tail -1 gpurun_out/$T/smoke.log
$S 300 gpurun_out/$T/prof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/p -o eng -- python3 tools/profile_engine.py --dtype fp32 --batches 12 || exit 1
f=$(find gpurun_out/$T/p -name "eng_kernel_trace.csv" | head -1)
python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/$T/ops.md > /dev/null 2>&1; grep "device time" gpurun_out/$T/ops.md
rm -f "$f"
$S 300 gpurun_out/$T/bench.log python bench.py --steps 20 --warmup 5 || exit 1
tail -1 gpurun_out/$T/bench.log | cut -c1-600
