#!/usr/bin/env bash
# Round-4 final engine: regenerate the fp32 tuning table for the default programs, then the whole GPU tier,
# smoke(), the fp32 kernel trace mapped to program ops (bs 32 and bs 1) and the driver-shaped bench.
# The new table comes back as gpurun_out/tuning/conv_tuning.json.  usage: scripts/gpurun/r4_final.sh TAG
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-r4final}
mkdir -p gpurun_out/$T gpurun_out/tuning
$S 900 gpurun_out/$T/tune.log python -u tools/tune_programs.py --dtypes fp32 --base data/tuning/conv_tuning.json --out gpurun_out/tuning/conv_tuning.json || exit 1
cp gpurun_out/tuning/conv_tuning.json data/tuning/conv_tuning.json
$S 900 gpurun_out/$T/pytest.log python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider || exit 1
tail -3 gpurun_out/$T/pytest.log
grep -q " failed" gpurun_out/$T/pytest.log && exit 1
$S 300 gpurun_out/$T/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
tail -1 gpurun_out/$T/smoke.log
for bs in 32 1; do
  $S 300 gpurun_out/$T/prof_$bs.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/p_$bs -o eng -- python3 tools/profile_engine.py --dtype fp32 --batch $bs --batches 12 || exit 1
  f=$(find gpurun_out/$T/p_$bs -name "eng_kernel_trace.csv" | head -1)
  python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/$T/ops_bs$bs.md > /dev/null 2>&1
  echo "bs=$bs: $(grep 'device time' gpurun_out/$T/ops_bs$bs.md)"
  find gpurun_out/$T/p_$bs -name "*kernel_stats.csv" -exec cp {} gpurun_out/$T/kernel_stats_bs$bs.csv \;
  rm -rf gpurun_out/$T/p_$bs
done
$S 600 gpurun_out/$T/bench.log python -u bench.py --steps 20 --warmup 5 || exit 1
grep '^{' gpurun_out/$T/bench.log | cut -c1-300
