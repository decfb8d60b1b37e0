#!/usr/bin/env bash
# ir_reg_x3 diagnosis: kernel time with phases switched off (ARENA_IR_REG_DBG), then one PMC pass
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-r5e}
mkdir -p gpurun_out/$T
for d in 0 1 2 4 7; do
  ARENA_IR_REG_DBG=$d $S 200 gpurun_out/$T/dbg$d.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/dbg$d -o t -- python3 tools/bench_irreg.py --crops 128 || exit 1
  f=$(find gpurun_out/$T/dbg$d -name "t_kernel_stats.csv" | head -1)
  echo "dbg=$d"; grep "ir_reg" "$f" | cut -d, -f1-4
  find gpurun_out/$T/dbg$d -name "*kernel_trace.csv" -delete
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/$T/pmc -o p -- python3 tools/bench_irreg.py --crops 128 --reps 3 > gpurun_out/$T/pmc.log 2>&1 || { echo "pmc rc=$?"; exit 1; }
f=$(find gpurun_out/$T/pmc -name "p_counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"]
    if "ir_reg" not in k and "ir_tile" not in k:
        continue
    agg[(k.split("(")[0], r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
per = collections.defaultdict(list)
for (k, d), c in agg.items():
    per[k].append(c)
for k, cs in per.items():
    keys = sorted(cs[0])
    print(k, {c: round(sum(x.get(c, 0) for x in cs) / len(cs) / 1e6, 2) for c in keys}, "(x1e6, mean over", len(cs), "dispatches)")
PY
