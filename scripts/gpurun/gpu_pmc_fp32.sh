#!/usr/bin/env bash
# fp32 engine hardware counters: one rocprofv3 --pmc pass per counter set over tools/profile_engine.py
# (kernel-trace + pmc only), then the per-op table (tools/analyze_pmc.py --dtype fp32).
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
T=${1:-pmc_fp32}
mkdir -p gpurun_out/$T
i=0
# every set carries GRBM_GUI_ACTIVE (GRBM block, its own slots): analyze_pmc.py checks each set's attribution by
# duration as well as by kernel name
for set in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/$T/s$i -o run -- \
    python3 tools/profile_engine.py --dtype fp32 --batches 4 > gpurun_out/$T/s$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "set $i failed rc=$rc"; exit 99; fi
done
# the op table (kernel names + un-profiled durations) comes from the caller's trace run: TIMES=<ops_bs32.md>
if [ -n "${TIMES:-}" ]; then
  python tools/analyze_pmc.py gpurun_out/$T/s*/run_counter_collection.csv --dtype fp32 --times "$TIMES" \
    --out gpurun_out/$T/ops.md > gpurun_out/$T/analyze.log 2>&1
  echo "analyze_pmc rc=$? $(grep -c '^- ' gpurun_out/$T/ops.md) problems"
  grep "Duration check" gpurun_out/$T/ops.md
fi
find gpurun_out/$T -name "*kernel_trace.csv" -delete
