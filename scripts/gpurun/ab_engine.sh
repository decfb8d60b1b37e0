#!/usr/bin/env bash
# A/B of an engine knob: GPU tests (optional), engine-only req/s per setting, fp32 per-op kernel tables.
# usage: scripts/gpurun/ab_engine.sh TAG VAR "v1 v2 ..." [pytest -k expression]
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=$1; VAR=$2; VALS=$3; K=${4:-}
mkdir -p gpurun_out/$T
if [ -n "$K" ]; then
  $S 600 gpurun_out/$T/pytest.log python -u -m pytest tests -m gpu -k "$K" -q --timeout 180 --timeout-method thread -p no:cacheprovider || exit 1
  grep -E "passed|failed" gpurun_out/$T/pytest.log | tail -2
  grep -q " failed" gpurun_out/$T/pytest.log && exit 1
fi
for v in $VALS; do
  env $VAR=$v $S 300 gpurun_out/$T/engine_$v.log python tools/engine_probe.py --batches 120 || exit 1
  grep "^engine" gpurun_out/$T/engine_$v.log
done
for v in $VALS; do
  for bs in 32 1; do
    env $VAR=$v $S 300 gpurun_out/$T/prof_${v}_$bs.log rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/p_${v}_$bs -o eng -- python3 tools/profile_engine.py --dtype fp32 --batch $bs --batches 12 || exit 1
    f=$(find gpurun_out/$T/p_${v}_$bs -name "eng_kernel_trace.csv" | head -1)
    env $VAR=$v python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/$T/ops_${v}_bs$bs.md > /dev/null 2>&1
    echo "$VAR=$v bs=$bs: $(grep 'device time' gpurun_out/$T/ops_${v}_bs$bs.md)"
    rm -rf gpurun_out/$T/p_${v}_$bs
  done
done
