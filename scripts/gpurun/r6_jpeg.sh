#!/usr/bin/env bash
# Compact vs dense JPEG payload under the pipelined engine loop: bit-exactness tests, engine req/s alternated, and a
# kernel trace of the pipelined loop per setting (which kernels grow when the IDCT reads the compact payload).
# usage: bash scripts/gpurun/r6_jpeg.sh TAG
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=$1
O=gpurun_out/$T
mkdir -p $O
$S 300 $O/pytest.log python -u -m pytest tests/test_jpeg_native_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " failed" $O/pytest.log && exit 1
for c in 1 0 1 0; do
  ARENA_JPEG_COMPACT=$c $S 300 $O/compact_$c.log python tools/engine_probe.py --inputs jpeg --batches 200 || exit 1
  echo "compact=$c: $(grep '^engine' $O/compact_$c.log)" | tee -a $O/summary.txt
done
for c in 1 0; do
  ARENA_JPEG_COMPACT=$c $S 300 $O/prof_$c.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$c -o eng -- python3 tools/engine_probe.py --inputs jpeg --batches 200 || exit 1
  f=$(find $O/p_$c -name "eng_kernel_stats.csv" | head -1)
  cp "$f" $O/kernel_stats_pipelined_$c.csv
  f=$(find $O/p_$c -name "eng_kernel_trace.csv" | head -1)
  python tools/busy_fraction.py "$f" --window-ms 500 > $O/busy_$c.txt 2>&1 || true
  cat $O/busy_$c.txt >> $O/summary.txt
  echo "compact=$c (traced): $(grep '^engine' $O/prof_$c.log)" | tee -a $O/summary.txt
  rm -rf $O/p_$c
done
