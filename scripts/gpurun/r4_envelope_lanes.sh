#!/usr/bin/env bash
# Round 4: the triton arm under the reference's 2-vCPU envelope (1 / 10 / 50 users), then the bs-1 latency of
# the Detect-head lanes (ARENA_HEAD_LANES 0 / 1; lanes run for buckets <= 2) from the driver-shaped bench's
# 1-user level.  usage: scripts/gpurun/r4_envelope_lanes.sh
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpurun/r4_protocol_batch.sh "triton 1,10,50 ENVELOPE=2 TAGSFX=_env2" || exit 1
mkdir -p gpurun_out/r4lanes_bs1
for v in 0 1; do
  ARENA_HEAD_LANES=$v scripts/gpurun/gpu_step.sh 300 gpurun_out/r4lanes_bs1/bench_$v.log python -u bench.py --steps 3 --warmup 2 \
    --latency-levels 1,10 --no-secondary-bf16 --no-secondary-inproc || exit 1
  echo "lanes=$v: $(grep -o '"levels": {[^}]*}[^}]*}' gpurun_out/r4lanes_bs1/bench_$v.log | head -1)"
done
