#!/usr/bin/env bash
# Round 4 engine experiments: 14x14 IR row bands (tests + engine A/B + per-op tables at bs 32 / 1), then the
# driver-shaped bench with blocking completion events.  usage: scripts/gpurun/r4_engine_ab.sh TAG
set -u
cd $GRAFT_REPO_ROOT
T=${1:-r4b}
bash scripts/gpurun/ab_engine.sh $T ARENA_IRX_PARTS "2 4 3" "ir_block_f32 and 14" || exit 1
ARENA_SYNC=blocking scripts/gpurun/gpu_step.sh 600 gpurun_out/$T/bench_blocking.log python -u bench.py --steps 20 --warmup 5 --latency-levels 1,10 --no-secondary-inproc --no-secondary-bf16 || exit 1
grep '^{' gpurun_out/$T/bench_blocking.log | cut -c1-200
