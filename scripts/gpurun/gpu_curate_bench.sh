set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
$S 300 gpurun_out/curate_fp32.log python tools/curate_workload.py --dtype fp32 --out data/synthetic_set/manifest_w0_n100.json || exit 1
cp data/synthetic_set/manifest_w0_n100.json gpurun_out/ || exit 1
$S 200 gpurun_out/decode_rate.log python tools/decode_rate.py --workers 1,8,15,24 || exit 1
$S 300 gpurun_out/bench_e2e2.log python bench.py --steps 60 --warmup 10 --bs1-requests 30 || exit 1
