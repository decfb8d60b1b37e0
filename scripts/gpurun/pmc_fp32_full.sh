#!/usr/bin/env bash
# fp32 engine counters, one rocprofv3 --pmc pass per set (kernel-trace + pmc only): instruction mix and waits,
# LDS conflicts and MFMA busy, HBM bytes (FETCH_SIZE and WRITE_SIZE in separate passes: 3 + 2 TCC counters),
# then the per-op table with achieved TB/s against a kernel-trace timing pass.  usage: pmc_fp32_full.sh TAG
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-pmc_full}
mkdir -p gpurun_out/$T
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/t -o eng -- python3 tools/profile_engine.py --dtype fp32 --batches 12 > gpurun_out/$T/t.log 2>&1 || { echo "trace failed"; exit 99; }
f=$(find gpurun_out/$T/t -name "eng_kernel_trace.csv" | head -1)
python tools/analyze_trace.py "$f" --dtype fp32 --replays 8 --out gpurun_out/$T/times.md > /dev/null 2>&1
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/$T/s$i -o run -- \
    python3 tools/profile_engine.py --dtype fp32 --batches 4 > gpurun_out/$T/s$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "set $i failed rc=$rc"; tail -5 gpurun_out/$T/s$i.log; exit 99; fi
done
python tools/analyze_pmc.py gpurun_out/$T/s*/run_counter_collection.csv --dtype fp32 --times gpurun_out/$T/times.md --out gpurun_out/$T/ops.md > /dev/null
find gpurun_out/$T -name "*kernel_trace.csv" -delete
find gpurun_out/$T -name "run_counter_collection.csv" -size +20M -delete
head -3 gpurun_out/$T/ops.md
