set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
$S 500 gpurun_out/split_tests.log python -u -m pytest tests/test_split_gpu.py tests/test_fp32_gpu.py tests/test_servers_gpu.py tests/test_pipeline_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
