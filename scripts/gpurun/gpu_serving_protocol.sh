#!/usr/bin/env bash
# The reference's closed-loop protocol levels (experiment.yaml: 1, 5, 10, 25, 50, 75, 100 users) on one MI355X
# for all three arms with the native HTTP layer, each arm at its best measured process layout; then the H1a-H1d
# evaluation over the combined rows (short phases: 5 s warm-up + 15 s measure).
set -euo pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1 ARENA_NATIVE_HTTP=1 LOG_LEVEL=WARNING ARENA_CROP_TRANSPORT=raw ARENA_FANOUT=batch
U=${USERS:-1,5,10,25,50,75,100}
O=gpurun_out/protocol
mkdir -p $O
ARENA_DECODE_PROCS=8 timeout -k 10 400 python scripts/serving_sweep.py --archs monolithic --users $U --procs 4 \
  --procs-per-gpu 1 --out $O/monolithic > $O/monolithic.log 2>&1
ARENA_DECODE_PROCS=4 timeout -k 10 400 python scripts/serving_sweep.py --archs triton --users $U --procs 4 \
  --procs-per-gpu 3 --out $O/triton > $O/triton.log 2>&1
ARENA_DECODE_PROCS=3 ARENA_CLS_PROCS_PER_GPU=2 timeout -k 10 400 python scripts/serving_sweep.py --archs microservices \
  --users $U --procs 4 --procs-per-gpu 3 --out $O/microservices > $O/microservices.log 2>&1
python - <<'PY'
import csv, json
from pathlib import Path
from inference_arena_amd.loadgen.hypotheses import evaluate
rows = []
for arch in ("monolithic", "triton", "microservices"):
    for r in csv.DictReader(open(f"gpurun_out/protocol/{arch}/{arch}_sweep.csv")):
        rows.append({"architecture": r["architecture"], "users": int(float(r["users"])),
                     **{k: float(r[k]) for k in ("p50_latency_ms", "p99_latency_ms", "throughput_rps",
                                                 "error_rate_percent")}})
Path("gpurun_out/protocol/hypotheses.json").write_text(json.dumps(evaluate(rows), indent=2, default=str) + "\n")
print(json.dumps(evaluate(rows), default=str))
PY
grep -h "users=" $O/*.log
