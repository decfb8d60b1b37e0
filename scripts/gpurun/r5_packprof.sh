#!/bin/bash
# JPEG stage per batch with coefficients packed into the batch DMA: kernel + memory-copy trace of the engine fed
# pinned coefficient sets (the HTTP path's inputs).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5packprof
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/r5packprof/p -o eng -- python3 tools/profile_engine.py --dtype fp32 --batches 12 --inputs jpeg > gpurun_out/r5packprof/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 gpurun_out/r5packprof/prof.log; exit 1; }
python tools/jpeg_stage_profile.py gpurun_out/r5packprof/p --out gpurun_out/r5packprof/jpeg_stage.md && cat gpurun_out/r5packprof/jpeg_stage.md
find gpurun_out/r5packprof/p -name "*kernel_trace.csv" -delete
true
