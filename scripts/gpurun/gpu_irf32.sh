set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
$S 400 gpurun_out/irf32_tests.log python -u -m pytest tests/test_fp32_gpu.py tests/test_split_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
mkdir -p gpurun_out/prof_irf
$S 300 gpurun_out/prof_irf/run.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_irf -o eng -- python3 tools/profile_engine.py --dtype fp32 --batches 12 || exit 1
f=$(find gpurun_out/prof_irf -name "eng_kernel_trace.csv" | head -1)
python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/prof_irf/ops.md > /dev/null 2>&1; tail -14 gpurun_out/prof_irf/ops.md
$S 300 gpurun_out/bench_e2e4.log python bench.py --steps 60 --warmup 10 --bs1-requests 30 || exit 1
