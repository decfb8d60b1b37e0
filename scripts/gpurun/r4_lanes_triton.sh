#!/usr/bin/env bash
# Round 4: Detect-head branches on side streams (ARENA_HEAD_LANES) A/B with its tests, then the triton arm at 100
# users with two model-server processes and with two slots per engine (bigger batches per engine).
set -u
cd $GRAFT_REPO_ROOT
bash scripts/gpurun/ab_engine.sh r4lanes ARENA_HEAD_LANES "0 1" "head_lanes" || exit 1
bash scripts/gpurun/r4_protocol_batch.sh "triton 100 PROCS_PER_GPU=2 TAGSFX=_ppg2" "triton 100 ARENA_SLOTS=2 TAGSFX=_slots2"
