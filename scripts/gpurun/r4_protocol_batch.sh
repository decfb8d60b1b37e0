#!/usr/bin/env bash
# Several protocol sweeps in one GPU call (boxes are scarce): each argument is "ARCH USERS [VAR=VAL ...]",
# run in order with scripts/gpurun/protocol.sh (TAG protocol_r4); RETUNE=1 first regenerates the fp32 tuning
# table on the box (scripts/gpurun/r4_retune.sh without its bench) so every sweep runs the tuned program.
# usage: scripts/gpurun/r4_protocol_batch.sh "monolithic 1,5,10" "triton 100 DECODE=4" ...
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tuning
if [ "${RETUNE:-0}" = "1" ]; then
  scripts/gpurun/gpu_step.sh 900 gpurun_out/tuning/tune.log python -u tools/tune_programs.py --dtypes fp32 \
    --base data/tuning/conv_tuning.json --out gpurun_out/tuning/conv_tuning.json || exit 1
  cp gpurun_out/tuning/conv_tuning.json data/tuning/conv_tuning.json
fi
for spec in "$@"; do
  set -- $spec
  arch=$1; users=$2; shift 2
  echo "== $arch $users $*"
  env "$@" bash scripts/gpurun/protocol.sh $arch $users protocol_r4 || { echo "sweep failed: $spec"; exit 1; }
done
