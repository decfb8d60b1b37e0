#!/usr/bin/env bash
# rocprofv3 kernel-trace + stats of a short bench run; summaries land in gpurun_out/prof.
# Serial slots by default (PCONC=1 profiles the concurrent executor) so per-op times are not inflated by overlap.
set -euo pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
python tools/build_ext.py > gpurun_out/build.log 2>&1
ARENA_CONCURRENT=${PCONC:-0} timeout -k 10 600 rocprofv3 --kernel-trace --stats ${PMARK:+--marker-trace} --output-format csv -d gpurun_out/prof -o bench -- \
  python3 bench.py --steps ${STEPS:-30} --warmup 5 --bs1-requests 0 > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err
cat gpurun_out/prof/bench.json
cp data/synthetic_set/*.json gpurun_out/ 2>/dev/null || true
find gpurun_out/prof -name "*stats*" | head
