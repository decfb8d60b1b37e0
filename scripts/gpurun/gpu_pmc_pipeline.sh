#!/usr/bin/env bash
# Counter sets over a short bench run (kernel-trace + pmc only), then the per-op table.
set -euo pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc2
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/pmc2/s$i -o run -- \
    python3 bench.py --steps 3 --warmup 2 --bs1-requests 0 > gpurun_out/pmc2/s$i.log 2>&1 || echo "set $i failed"
done
python tools/analyze_pmc.py gpurun_out/pmc2/s*/run_counter_collection.csv --out gpurun_out/pmc2/ops.md > /dev/null
head -5 gpurun_out/pmc2/ops.md
