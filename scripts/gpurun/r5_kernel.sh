#!/usr/bin/env bash
# Kernel iteration: GPU tests of the touched kernels, a rocprofv3 kernel-trace of a kernel microbenchmark, then
# (PROFILE=1) the fp32 engine op tables and (BENCH=1) the driver-shaped bench.
# usage: scripts/gpurun/r5_kernel.sh TAG "pytest targets" "bench tool + args" [-- bench args]
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=$1; TESTS=$2; TOOL=$3
shift 3
[ $# -gt 0 ] && [ "$1" = "--" ] && shift
mkdir -p gpurun_out/$T
if [ -n "$TESTS" ]; then
  $S 900 gpurun_out/$T/pytest.log python -u -m pytest $TESTS -x -v --timeout 180 --timeout-method thread -p no:cacheprovider || exit 1
  grep -E "passed|failed|error" gpurun_out/$T/pytest.log | tail -3
  grep -q " failed\| error" gpurun_out/$T/pytest.log && exit 1
fi
if [ -n "$TOOL" ]; then
  $S 300 gpurun_out/$T/tool.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/tool -o tool -- python3 $TOOL || exit 1
  f=$(find gpurun_out/$T/tool -name "tool_kernel_stats.csv" | head -1)
  [ -n "$f" ] && cut -d, -f1-8 "$f" | head -20
  find gpurun_out/$T/tool -name "*kernel_trace.csv" -delete
fi
if [ "${PROFILE:-0}" = "1" ]; then
  $S 300 gpurun_out/$T/prof_rgb.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof_rgb -o eng -- python3 tools/profile_engine.py --dtype fp32 --batches 12 || exit 1
  f=$(find gpurun_out/$T/prof_rgb -name "eng_kernel_trace.csv" | head -1)
  python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/$T/ops_bs32.md > /dev/null 2>&1; tail -16 gpurun_out/$T/ops_bs32.md
  rm -f "$f"
fi
if [ "${JPEGPROF:-0}" = "1" ]; then
  $S 300 gpurun_out/$T/prof_jpeg.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof_jpeg -o eng -- python3 tools/profile_engine.py --dtype fp32 --batches 12 --inputs jpeg || exit 1
  python tools/jpeg_stage_profile.py gpurun_out/$T/prof_jpeg --out gpurun_out/$T/jpeg_stage.md || true
  find gpurun_out/$T/prof_jpeg -name "*kernel_trace.csv" -size +2M -delete
fi
if [ "${BENCH:-0}" = "1" ]; then
  $S 900 gpurun_out/$T/bench.log python -u bench.py "$@" || exit 1
  grep '^{' gpurun_out/$T/bench.log | tail -1 > gpurun_out/$T/bench.json
  cut -c1-1800 gpurun_out/$T/bench.json
fi
