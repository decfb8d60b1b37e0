#!/usr/bin/env bash
# Copy the judged part of a protocol sweep (per-level summary JSONs, per-call sweep CSVs, the sweep logs) from
# gpurun_out/<tag>/ into profiles/<tag>/ and render the tables: mean ± sd per level (tools/protocol_table.py) and
# the hypothesis / RQ analysis of one engine (scripts/analyze_results.py).  Per-request CSVs and server logs stay
# in gpurun_out/.   usage: tools/collect_protocol.sh TAG [deploy_time.json]
set -eu
T=$1; DEPLOY=${2:-}
SRC=gpurun_out/$T; DST=profiles/$T
mkdir -p $DST
args=()
for d in $SRC/*/; do
  a=$(basename $d)
  mkdir -p $DST/$a
  cp $d/*_summary.json $DST/$a/ 2>/dev/null || true
  cp $d/*_sweep_L*.csv $d/*_sweep_all.csv $DST/$a/ 2>/dev/null || true
  cp $d/sweep.log $DST/$a/ 2>/dev/null || true
  label=$a
  [ "$a" = "microservices" ] && label="microservices, reference mode"
  [ "$a" = "microservices_device" ] && label="microservices, device mode"
  [ "$a" = "triton_tensor" ] && label="triton, reference-shaped tensor mode"
  [ "$a" = "triton_tensor8" ] && label="triton, reference-shaped tensor mode, 8 gateway processes"
  args+=("$DST/$a:$label")
done
python tools/protocol_table.py "${args[@]}" > $DST/table.md
extra=()
if [ -n "$DEPLOY" ]; then cp $DEPLOY $DST/deploy_time.json; extra=(--deploy $DST/deploy_time.json); fi
python scripts/analyze_results.py $DST/*/*_sweep_L*.csv --gpus 1 --out $DST/analysis "${extra[@]}" > /dev/null
echo "$DST/table.md $DST/analysis/summary.md"
