#!/usr/bin/env bash
# Round 4 closing evidence: the 2-rank rehearsal of the driver's multi-GPU bench (per-rank and shared front) and
# the fp32 program's hardware counters (instruction mix, MFMA busy, LDS conflicts, HBM bytes per op).
set -u
cd $GRAFT_REPO_ROOT
bash scripts/gpurun/rehearse_2rank.sh r4rehearse2 || exit 1
bash scripts/gpurun/gpu_pmc_fp32.sh r4pmc || exit 1
