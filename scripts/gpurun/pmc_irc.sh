#!/usr/bin/env bash
# hardware counters of the fused fp32 IR kernels on MobileNetV2 block shapes (tools/bench_irc.py),
# one rocprofv3 --pmc pass per counter set; prints per-kernel averages
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
export ARENA_IRC_F32=1
T=${1:-pmc_irc}
mkdir -p gpurun_out/$T
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES" \
           "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/$T/s$i -o run -- \
    python3 tools/bench_irc.py --small --reps 3 > gpurun_out/$T/s$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "set $i failed rc=$rc"; tail -5 gpurun_out/$T/s$i.log; exit 99; fi
done
find gpurun_out/$T -name "*kernel_trace.csv" -delete
python3 - "$T" <<'PY'
import csv, glob, sys, collections
T = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"gpurun_out/{T}/s*/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "ir_x3" not in k and "ir_f32" not in k:
            continue
        acc[k[k.find("<"):k.find(">") + 1] or k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: f"{sum(v) / len(v):.3g}" for c, v in sorted(d.items())})
PY
