#!/usr/bin/env bash
# 2-rank rehearsal of the driver's multi-GPU bench command on a 1-GPU box: bench.py self-launches 2 ranks over
# gloo, both on GPU 0 (ARENA_SHARED_GPU=1), HTTP path, weights verified, max over ranks.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp ARENA_SHARED_GPU=1 ARENA_DIST_BACKEND=gloo
S=scripts/gpurun/gpu_step.sh
T=${1:-rehearse2}
mkdir -p gpurun_out/$T
$S 600 gpurun_out/$T/bench2.log python bench.py --gpus 2 --steps 10 --warmup 3 --no-secondary-bf16 --no-secondary-inproc || exit 1
grep -v "^\[Gloo\]" gpurun_out/$T/bench2.log | tail -4 | cut -c1-900
# the node-level front door: both ranks bind one port (SO_REUSEPORT), rank 0's load generator drives it
$S 600 gpurun_out/$T/bench2_shared.log python bench.py --gpus 2 --steps 10 --warmup 3 --front shared --no-secondary-bf16 --no-secondary-inproc || exit 1
grep -v "^\[Gloo\]" gpurun_out/$T/bench2_shared.log | tail -4 | cut -c1-900
