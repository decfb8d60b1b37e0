#!/usr/bin/env bash
# Engine req/s (HTTP path's device inputs) per environment configuration, REPS rounds interleaved.
# usage: REPS=2 bash scripts/gpurun/env_sweep.sh TAG "ARENA_STAGGER=0.25" "ARENA_STAGGER=0.2,0.45+ARENA_SLOTS=5" ...
#        ('+' separates the assignments of one configuration)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
n=0
for r in $(seq 1 ${REPS:-2}); do
  i=0
  for cfg in "$@"; do
    i=$((i + 1))
    envs=$(echo "$cfg" | tr '+' ' ')
    env $envs $S 300 $O/e_${i}_$r.log python tools/engine_probe.py --inputs jpeg --batches ${BATCHES:-300} || exit 1
    echo "[$cfg] run $r: $(grep '^engine' $O/e_${i}_$r.log | cut -d'(' -f1)" | tee -a $O/summary.txt
  done
done
