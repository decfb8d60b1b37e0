#!/usr/bin/env bash
# Hardware counters for selected conv layers (kernel-trace + pmc only; no sys/runtime trace).
set -euo pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1 || true
OPS=${OPS:-13,37,40,51,53,23}
for set in "FETCH_SIZE WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE"; do
  tag=$(echo $set | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/pmc/$tag -o run -- \
    python3 tools/bench_convs.py --impls 2 --iters 3 --ops $OPS > gpurun_out/pmc/$tag.log 2>&1 || echo "counter set '$set' failed"
done
ls -R gpurun_out/pmc | head -50
