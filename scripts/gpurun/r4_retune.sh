#!/usr/bin/env bash
# Regenerate the fp32 entries of the conv tuning table after a program change (engine/tuning.py), then a
# driver-shaped bench against the new table.  The table comes back as gpurun_out/tuning/conv_tuning.json.
# usage: scripts/gpurun/r4_retune.sh TAG
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-r4e}
mkdir -p gpurun_out/$T gpurun_out/tuning
$S 900 gpurun_out/$T/tune.log python -u tools/tune_programs.py --dtypes fp32 --base data/tuning/conv_tuning.json --out gpurun_out/tuning/conv_tuning.json || exit 1
cp gpurun_out/tuning/conv_tuning.json data/tuning/conv_tuning.json
$S 600 gpurun_out/$T/bench.log python -u bench.py --steps 20 --warmup 5 || exit 1
grep '^{' gpurun_out/$T/bench.log | cut -c1-400
