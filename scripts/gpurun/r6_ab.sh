#!/usr/bin/env bash
# Round-6 A/B of the defaults, all in one box so box-to-box variance cancels:
#   1. compact vs dense JPEG payload (ARENA_JPEG_COMPACT): engine req/s on the HTTP path's device inputs, and the
#      per-kernel time of the reconstruction kernels (rocprofv3 --stats)
#   2. shipped tuning table vs a candidate (TUNING=path): engine req/s, alternated A B A B
#   3. executor concurrency (ARENA_SLOTS x ARENA_CONCURRENCY) with GPU_MAX_HW_QUEUES=8 (SWEEP=configs, optional)
# usage: TUNING=profiles/r6hr/conv_tuning.json SWEEP=4x3,6x4 bash scripts/gpurun/r6_ab.sh TAG
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=$1
O=gpurun_out/$T
mkdir -p $O
for c in 1 0 1 0; do
  ARENA_JPEG_COMPACT=$c $S 300 $O/compact_$c.log python tools/engine_probe.py --inputs jpeg --batches 200 || exit 1
  echo "compact=$c: $(grep '^engine' $O/compact_$c.log)" | tee -a $O/summary.txt
done
for c in 1 0; do
  ARENA_JPEG_COMPACT=$c $S 300 $O/prof_$c.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$c -o eng -- python3 tools/profile_engine.py --inputs jpeg --batch 32 --batches 20 || exit 1
  f=$(find $O/p_$c -name "eng_kernel_stats.csv" | head -1)
  cp "$f" $O/kernel_stats_compact_$c.csv
  grep -i "jpeg\|idct" $O/kernel_stats_compact_$c.csv | cut -c1-200 | tee -a $O/summary.txt
  grep -E "MB|ms/batch" $O/prof_$c.log | tee -a $O/summary.txt
  rm -rf $O/p_$c
done
if [ -n "${TUNING:-}" ]; then
  for r in 1 2; do
    $S 300 $O/tune_shipped_$r.log python tools/engine_probe.py --inputs jpeg --batches 200 || exit 1
    echo "shipped table: $(grep '^engine' $O/tune_shipped_$r.log)" | tee -a $O/summary.txt
    ARENA_TUNING_FILE=$TUNING $S 300 $O/tune_cand_$r.log python tools/engine_probe.py --inputs jpeg --batches 200 || exit 1
    echo "candidate $TUNING: $(grep '^engine' $O/tune_cand_$r.log)" | tee -a $O/summary.txt
  done
fi
if [ -n "${SWEEP:-}" ]; then
  GPU_MAX_HW_QUEUES=8 $S 600 $O/sweep.log python tools/sweep_concurrency.py --batches 120 --configs $SWEEP || exit 1
  tail -n 20 $O/sweep.log | tee -a $O/summary.txt
fi
