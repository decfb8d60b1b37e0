#!/usr/bin/env bash
# hardware counters of fp32 conv kernels on single layer shapes (tools/bench_x3g.py), one rocprofv3 --pmc pass
# per counter set; prints per-kernel averages.  usage: scripts/gpurun/pmc_x3g.sh TAG IMPLS SHAPES
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-pmc_x3g}
IMPLS=${2:-115}
SHAPES=${3:-det_s2_64}
mkdir -p gpurun_out/$T
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES" \
           "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/$T/s$i -o run -- \
    python3 tools/bench_x3g.py --impls $IMPLS --shapes $SHAPES --iters 5 > gpurun_out/$T/s$i.log 2>&1
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
        if "arena::" not in k or "direct" in k:
            continue
        name = k.split("(")[0].replace("void arena::", "")
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    w = max(m.get("SQ_WAVES", 1), 1)
    busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(m.get("GRBM_GUI_ACTIVE", 1) / 8 * 1024, 1) * 100
    wc = max(m.get("SQ_WAVE_CYCLES", 1), 1)
    print(f"{k}: waves {w:.0f} valu/wave {m.get('SQ_INSTS_VALU', 0) / w:.0f} mfma/wave {m.get('SQ_INSTS_MFMA', 0) / w:.0f} "
          f"lds/wave {m.get('SQ_INSTS_LDS', 0) / w:.0f} wait_any {m.get('SQ_WAIT_ANY', 0) / wc * 100:.0f}% "
          f"wait_inst {m.get('SQ_WAIT_INST_ANY', 0) / wc * 100:.0f}% lds_conflict "
          f"{m.get('SQ_LDS_BANK_CONFLICT', 0) / max(m.get('SQ_LDS_IDX_ACTIVE', 1), 1) * 100:.0f}% mfma_busy {busy:.0f}% "
          f"fetch {m.get('FETCH_SIZE', 0) / 1024:.1f} MB write {m.get('WRITE_SIZE', 0) / 1024:.1f} MB")
PY
