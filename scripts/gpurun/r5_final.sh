#!/usr/bin/env bash
# Round-5 closing evidence, in two calls (each within one gpurun limit):
#   r5_final.sh tier TAG   the whole GPU test tier, smoke() and the driver-shaped bench (no flags: the driver's
#                          defaults)
#   r5_final.sh prof TAG   fp32 kernel traces mapped to program ops (bs 32 and bs 1), the JPEG stage of the HTTP
#                          inputs, and the hardware counters per op with durations (analyze_pmc.py --times)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
MODE=$1; T=${2:-r5final}
mkdir -p gpurun_out/$T
if [ "$MODE" = "tier" ]; then
  $S 1000 gpurun_out/$T/pytest.log python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider || exit 1
  tail -3 gpurun_out/$T/pytest.log
  grep -q " failed\| error" gpurun_out/$T/pytest.log && exit 1
  $S 300 gpurun_out/$T/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
  tail -1 gpurun_out/$T/smoke.log
  $S 900 gpurun_out/$T/bench.log python -u bench.py || exit 1
  grep '^{' gpurun_out/$T/bench.log | tail -1 > gpurun_out/$T/bench.json
  cut -c1-400 gpurun_out/$T/bench.json
  exit 0
fi
for bs in 32 1; do
  $S 300 gpurun_out/$T/prof_$bs.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/p_$bs -o eng -- python3 tools/profile_engine.py --dtype fp32 --batch $bs --batches 12 || exit 1
  f=$(find gpurun_out/$T/p_$bs -name "eng_kernel_trace.csv" | head -1)
  python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/$T/ops_bs$bs.md > /dev/null 2>&1
  echo "bs=$bs: $(grep 'device time' gpurun_out/$T/ops_bs$bs.md)"
  find gpurun_out/$T/p_$bs -name "*kernel_stats.csv" -exec cp {} gpurun_out/$T/kernel_stats_bs$bs.csv \;
  rm -rf gpurun_out/$T/p_$bs
done
$S 300 gpurun_out/$T/prof_jpeg.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof_jpeg -o eng -- python3 tools/profile_engine.py --dtype fp32 --batches 12 --inputs jpeg || exit 1
python tools/jpeg_stage_profile.py gpurun_out/$T/prof_jpeg --out gpurun_out/$T/jpeg_stage.md || true
find gpurun_out/$T/prof_jpeg -name "*kernel_trace.csv" -delete
bash scripts/gpurun/gpu_pmc_fp32.sh $T/pmc || exit 1
python tools/analyze_pmc.py gpurun_out/$T/pmc/s*/run_counter_collection.csv --dtype fp32 --times gpurun_out/$T/ops_bs32.md --out gpurun_out/$T/ops_pmc.md > /dev/null
head -8 gpurun_out/$T/ops_pmc.md | cut -c1-300
