#!/bin/bash
# HEAD check after packing JPEG coefficients into the batch DMA by default: GPU tier, smoke, bench, then one 60 s run
# of the Triton and monolithic arms at 100 users (CPU per process, RSS) under gpurun_out/protocol_r5/<arch>_pack.
set -u
cd $GRAFT_REPO_ROOT
bash scripts/gpurun/r5_final.sh tier r5final4 || exit 1
RUNS=1 TAGSFX=_pack bash scripts/gpurun/r5_sweep.sh triton 100 || exit 1
RUNS=1 TAGSFX=_pack bash scripts/gpurun/r5_sweep.sh monolithic 100 || exit 1
