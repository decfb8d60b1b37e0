#!/usr/bin/env bash
set -uo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for env in "" "DEBUG_HIP_GRAPH_PACKET_CAPTURE=0" "HIP_FORCE_DEV_KERNARG=0"; do
  echo "== env: $env"
  env $env timeout -k 10 120 python scripts/probe_kernargs.py 2>&1 | grep -v amdgpu.ids
done
