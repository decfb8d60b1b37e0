#!/usr/bin/env bash
# Round-6 kernel evidence in one call: fp32 kernel traces mapped to program ops (bs 32, and bs 1 with BS1=1), then
# the hardware counters per op (gpu_pmc_fp32.sh: one pass per set, attribution checked by analyze_pmc.py against
# the bs-32 op table).
#   r6_prof.sh TAG
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-r6prof}
mkdir -p gpurun_out/$T
BSS="32"
[ "${BS1:-0}" = "1" ] && BSS="32 1"
for bs in $BSS; do
  $S 300 gpurun_out/$T/prof_$bs.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/p_$bs -o eng -- python3 tools/profile_engine.py --dtype fp32 --batch $bs --batches 12 || exit 1
  f=$(find gpurun_out/$T/p_$bs -name "eng_kernel_trace.csv" | head -1)
  python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/$T/ops_bs$bs.md > /dev/null 2>&1
  echo "bs=$bs: $(grep 'device time' gpurun_out/$T/ops_bs$bs.md)"
  find gpurun_out/$T/p_$bs -name "*kernel_stats.csv" -exec cp {} gpurun_out/$T/kernel_stats_bs$bs.csv \;
  rm -rf gpurun_out/$T/p_$bs
done
if [ "${PMC:-1}" = "1" ]; then
  TIMES=gpurun_out/$T/ops_bs32.md bash scripts/gpurun/gpu_pmc_fp32.sh $T/pmc || exit 1
fi
