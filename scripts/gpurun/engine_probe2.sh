set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
mkdir -p gpurun_out/probe2
for cfg in "4 3" "4 2" "4 4" "5 3" "3 3"; do
  set -- $cfg
  ARENA_SLOTS=$1 ARENA_CONCURRENCY=$2 $S 200 gpurun_out/probe2/e_$1_$2.log python tools/engine_probe.py --batches 300 || exit 1
  grep engine gpurun_out/probe2/e_$1_$2.log | tail -1
done
