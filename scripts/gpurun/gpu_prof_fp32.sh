# fp32 engine profile: rocprofv3 kernel trace of tools/profile_engine.py -> per-op table (analyze_trace.py)
# usage: scripts/gpurun/gpu_prof_fp32.sh TAG
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-prof}
mkdir -p gpurun_out/$T
$S 300 gpurun_out/$T/run.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T -o eng -- python3 tools/profile_engine.py --dtype fp32 --batches 12 || exit 1
f=$(find gpurun_out/$T -name "eng_kernel_trace.csv" | head -1)
python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/$T/ops.md > /dev/null 2>&1; tail -14 gpurun_out/$T/ops.md
rm -f "$f"
