#!/usr/bin/env bash
# A/B of the host-side defaults on one box: (decode workers, HTTP I/O threads), alternated twice.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
mkdir -p gpurun_out/hostab
for rep in 1 2; do
  for cfg in "10 4" "11 2" "10 2"; do
    set -- $cfg
    $S 300 gpurun_out/hostab/w$1_t$2_$rep.log python bench.py --steps 20 --warmup 5 --no-secondary-bf16 --no-secondary-inproc --latency-levels '' --decode-workers $1 --http-threads $2 || exit 1
    echo "W=$1 T=$2 rep $rep: $(grep -o '"value": [0-9.]*' gpurun_out/hostab/w$1_t$2_$rep.log | tail -1)"
  done
done
