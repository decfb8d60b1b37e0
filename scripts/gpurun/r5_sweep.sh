#!/usr/bin/env bash
# Round 5 protocol sweep on one engine (the round-5 HEAD): ARCH at the given user levels, 60 s x 3 runs per level
# (10 s warm-up, 2 s cooldown), summaries under gpurun_out/protocol_r5/<arch>[suffix]/.  Arm B runs in the
# reference's mode (PIL JPEG q95 crops, one Classify RPC per crop under asyncio.gather) unless TRANSPORT / FANOUT
# say otherwise; the Triton arm's gateway is the native proxy to the model server's KServe REST endpoint.
# usage: scripts/gpurun/r5_sweep.sh ARCH LEVELS   (e.g. monolithic 1,5,10,25)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
WARMUP=${WARMUP:-10} MEASURE=${MEASURE:-60} RUNS=${RUNS:-3} COOLDOWN=${COOLDOWN:-2} \
  bash scripts/gpurun/protocol.sh "$1" "$2" protocol_r5 || exit 1
# the next call for the same arm rewrites <arch>_sweep.csv: keep this call's rows under a per-level-set name
O=gpurun_out/protocol_r5/$1${TAGSFX:-}
L=$(echo "$2" | tr ',' '_')
[ -f $O/$1_sweep.csv ] && cp $O/$1_sweep.csv $O/$1_sweep_L$L.csv
true
