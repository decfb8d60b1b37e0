#!/usr/bin/env bash
# Round-6 kernel iteration in one call: the touched kernels' GPU tests, a standalone microbenchmark
# (tools/bench_x3g.py SHAPES x IMPLS), a retune of the fp32 pipeline's bucket-32 (and bucket-1) conv choices
# against a copy of the shipped table, and the fp32 op table with the retuned program.
#   r6_kernel.sh TAG "pytest args" "bench_x3g args"
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=$1; TESTS=$2; MB=$3
mkdir -p gpurun_out/$T
if [ -n "$TESTS" ]; then
  $S 900 gpurun_out/$T/pytest.log python -u -m pytest $TESTS -x -q --timeout 180 --timeout-method thread -p no:cacheprovider || exit 1
  tail -2 gpurun_out/$T/pytest.log
  grep -q " failed\| error" gpurun_out/$T/pytest.log && exit 1
fi
if [ -n "${TESTS2:-}" ]; then
  $S 900 gpurun_out/$T/pytest2.log python -u -m pytest $TESTS2 -x -q --timeout 180 --timeout-method thread -p no:cacheprovider || exit 1
  tail -2 gpurun_out/$T/pytest2.log
  grep -q " failed\| error" gpurun_out/$T/pytest2.log && exit 1
fi
if [ -n "${REPRO:-}" ]; then  # HIP-only retention repro (csrc/tests/hip_retention_repro.cpp), each mode
  for m in $REPRO; do
    $S 240 gpurun_out/$T/repro_$m.log tools/bin/hip_retention_repro $m 6000 32 || exit 1
    tail -1 gpurun_out/$T/repro_$m.log
  done
fi
if [ -n "$MB" ]; then
  $S 600 gpurun_out/$T/mb.log python -u tools/bench_x3g.py $MB || exit 1
  grep -v "^\[gpu_step\]" gpurun_out/$T/mb.log | cut -c1-2000
fi
if [ "${RETUNE:-1}" = "1" ]; then
  $S 900 gpurun_out/$T/tune.log python -u tools/tune_programs.py --dtypes fp32 --kinds pipeline --buckets ${TUNE_BUCKETS:-1,32} --base data/tuning/conv_tuning.json --out gpurun_out/$T/conv_tuning.json || exit 1
  tail -2 gpurun_out/$T/tune.log
  export ARENA_TUNING_FILE=gpurun_out/$T/conv_tuning.json
fi
for bs in ${PROF_BS:-32}; do
  $S 300 gpurun_out/$T/prof_$bs.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/p -o eng -- python3 tools/profile_engine.py --dtype fp32 --batch $bs --batches 12 || exit 1
  f=$(find gpurun_out/$T/p -name "eng_kernel_trace.csv" | head -1)
  python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/$T/ops_bs$bs.md > /dev/null 2>&1
  echo "bs $bs: $(grep 'device time' gpurun_out/$T/ops_bs$bs.md)"
  rm -rf gpurun_out/$T/p
done
if [ "${BENCH:-0}" = "1" ]; then
  $S 900 gpurun_out/$T/bench.log python -u bench.py --steps 20 --warmup 5 --latency-levels "" --no-secondary-inproc --no-secondary-bf16 || exit 1
  grep '^{' gpurun_out/$T/bench.log | tail -1 | cut -c1-600
fi
