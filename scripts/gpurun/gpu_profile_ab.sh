#!/usr/bin/env bash
# A/B kernel-trace profiles of bench.py under two environment settings (serial executor):
#   ENV_A="ARENA_FUSE_STEM=0" ENV_B="ARENA_FUSE_STEM=1" bash scripts/gpurun/gpu_profile_ab.sh
set -euo pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
python tools/build_ext.py > gpurun_out/build.log 2>&1
for tag in A B; do
  var="ENV_$tag"
  ( export ARENA_CONCURRENT=${PCONC:-0} ${!var}
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab/$tag -o t -- \
      python3 bench.py --steps ${STEPS:-20} --warmup 5 --bs1-requests 0 > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err )
  ( export ${!var}; python tools/analyze_trace.py $(find gpurun_out/ab/$tag -name "*kernel_trace.csv" | head -1) --out gpurun_out/ab/$tag.md > /dev/null )
  echo "$tag (${!var}): $(tail -c 400 gpurun_out/ab/$tag.json | grep -o '"value": [0-9.]*')"
done
