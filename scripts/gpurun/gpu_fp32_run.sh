set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
$S 400 gpurun_out/fp32_tests.log python -u -m pytest tests/test_fp32_gpu.py tests/test_programs_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
$S 300 gpurun_out/bench_fp32.log python bench.py --steps 30 --warmup 5 --bs1-requests 20 || exit 1
