#!/usr/bin/env bash
# Kernel changes of the round (stem LDS strides, JPEG colour kernel): their GPU tests, then the fp32 op table at
# batch 32 and the JPEG stage profile.  usage: scripts/gpurun/r5_validate.sh TAG
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-r5v}
mkdir -p gpurun_out/$T
$S 600 gpurun_out/$T/pytest.log python -u -m pytest tests/test_fp32_gpu.py -k stem tests/test_kernels_gpu.py -k "stem" tests/test_jpeg_native_gpu.py tests/test_headline_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
grep -E "passed|failed|error" gpurun_out/$T/pytest.log | tail -2
grep -q " failed\| error" gpurun_out/$T/pytest.log && exit 1
$S 300 gpurun_out/$T/prof_32.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/p_32 -o eng -- python3 tools/profile_engine.py --dtype fp32 --batch 32 --batches 12 || exit 1
f=$(find gpurun_out/$T/p_32 -name "eng_kernel_trace.csv" | head -1)
python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/$T/ops_bs32.md > /dev/null 2>&1
grep "device time\| 1 | stem" gpurun_out/$T/ops_bs32.md
rm -rf gpurun_out/$T/p_32
$S 300 gpurun_out/$T/prof_jpeg.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof_jpeg -o eng -- python3 tools/profile_engine.py --dtype fp32 --batches 12 --inputs jpeg || exit 1
python tools/jpeg_stage_profile.py gpurun_out/$T/prof_jpeg --out gpurun_out/$T/jpeg_stage.md | head -5 || true
find gpurun_out/$T/prof_jpeg -name "*kernel_trace.csv" -delete
true
