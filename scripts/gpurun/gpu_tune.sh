set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
$S 500 gpurun_out/tune.log python tools/tune_programs.py --out gpurun_out/conv_tuning.json || exit 1
$S 300 gpurun_out/tune_test.log python -u -m pytest tests/test_kernels_gpu.py -x -q -k "autotune" --timeout 200 --timeout-method thread -p no:cacheprovider || exit 1
