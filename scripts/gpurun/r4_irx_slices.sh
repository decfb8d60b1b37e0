#!/usr/bin/env bash
# Round 4: hidden-sliced whole-map IR blocks (14x14 and the 7x7 tail) — tests, engine A/B and per-op tables.
# usage: scripts/gpurun/r4_irx_slices.sh TAG
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-r4d}
mkdir -p gpurun_out/$T
$S 600 gpurun_out/$T/pytest.log python -u -m pytest tests -m gpu -k "hidden_slices or (ir_block_f32 and 14) or pipeline_matches_reference or split_programs" -q --timeout 180 --timeout-method thread -p no:cacheprovider || exit 1
grep -E "passed|failed" gpurun_out/$T/pytest.log | tail -1
grep -q " failed" gpurun_out/$T/pytest.log && exit 1
for cfg in "1 0" "6 0" "6 1"; do
  set -- $cfg
  tag=s$1t$2
  ARENA_IRX_SLICES=$1 ARENA_IRX_TAIL=$2 $S 300 gpurun_out/$T/engine_$tag.log python tools/engine_probe.py --batches 120 || exit 1
  grep "^engine" gpurun_out/$T/engine_$tag.log | head -1
  for bs in 32 1; do
    ARENA_IRX_SLICES=$1 ARENA_IRX_TAIL=$2 $S 300 gpurun_out/$T/prof_${tag}_$bs.log rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/p_${tag}_$bs -o eng -- python3 tools/profile_engine.py --dtype fp32 --batch $bs --batches 12 || exit 1
    f=$(find gpurun_out/$T/p_${tag}_$bs -name "eng_kernel_trace.csv" | head -1)
    python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/$T/ops_${tag}_bs$bs.md > /dev/null 2>&1
    echo "$tag bs=$bs: $(grep 'device time' gpurun_out/$T/ops_${tag}_bs$bs.md)"
    rm -rf gpurun_out/$T/p_${tag}_$bs
  done
done
