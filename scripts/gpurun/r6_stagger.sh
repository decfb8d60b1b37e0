#!/usr/bin/env bash
# Staggered launch sweep (ARENA_STAGGER) x JPEG payload (ARENA_JPEG_COMPACT): engine req/s on the HTTP path's
# device inputs, each setting twice, interleaved.
# usage: VALS="0 0.2 0.33 0.5" bash scripts/gpurun/r6_stagger.sh TAG
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=$1
O=gpurun_out/$T
mkdir -p $O
VALS=${VALS:-"0 0.2 0.33 0.5"}
for r in 1 2; do
  for c in 1 0; do
    for v in $VALS; do
      ARENA_STAGGER=$v ARENA_JPEG_COMPACT=$c $S 300 $O/e_${v}_${c}_$r.log python tools/engine_probe.py --inputs jpeg --batches 300 || exit 1
      echo "stagger=$v compact=$c run $r: $(grep '^engine' $O/e_${v}_${c}_$r.log | cut -d'(' -f1)" | tee -a $O/summary.txt
    done
  done
done
