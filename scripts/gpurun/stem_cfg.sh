#!/usr/bin/env bash
# fused fp32 stem configurations: numerics tests, then an engine kernel trace per (TH, NW), op 1 time each.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-stemcfg}
mkdir -p gpurun_out/$T
$S 300 gpurun_out/$T/tests.log python -u -m pytest tests/test_fp32_gpu.py -x -q -k "stem_s2" --timeout 200 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" gpurun_out/$T/tests.log && ! grep -q "failed" gpurun_out/$T/tests.log || { echo "tests failed"; tail -30 gpurun_out/$T/tests.log; exit 1; }
for cfg in ${CFGS:-4:2 4:4 8:4}; do
  th=${cfg%:*}; nw=${cfg#*:}
  ARENA_STEM_X3_TH=$th ARENA_STEM_X3_NW=$nw $S 300 gpurun_out/$T/prof_$th$nw.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/p$th$nw -o eng -- python3 tools/profile_engine.py --dtype fp32 --batches 12 || exit 1
  f=$(find gpurun_out/$T/p$th$nw -name "eng_kernel_trace.csv" | head -1)
  python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/$T/ops_$th$nw.md > /dev/null 2>&1
  echo "TH=$th NW=$nw: $(sed -n 4p gpurun_out/$T/ops_$th$nw.md | cut -d'|' -f5,8) $(grep 'device time' gpurun_out/$T/ops_$th$nw.md)"
  rm -f "$f"
done
