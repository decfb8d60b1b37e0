set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
$S 300 gpurun_out/curate_fp32.log python tools/curate_workload.py --dtype fp32 --out data/synthetic_set/manifest_w0_n100.json || exit 1
cp data/synthetic_set/manifest_w0_n100.json gpurun_out/ || exit 1
$S 400 gpurun_out/fp32_tests2.log python -u -m pytest tests/test_fp32_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
mkdir -p gpurun_out/prof_lds
$S 300 gpurun_out/prof_lds/run.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lds -o eng -- python3 tools/profile_engine.py --dtype fp32 --batches 12 || exit 1
f=$(find gpurun_out/prof_lds -name "eng_kernel_trace.csv" | head -1)
python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/prof_lds/ops.md > /dev/null 2>&1; tail -14 gpurun_out/prof_lds/ops.md
$S 300 gpurun_out/bench_e2e3.log python bench.py --steps 60 --warmup 10 --bs1-requests 30 || exit 1
