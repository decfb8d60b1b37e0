#!/usr/bin/env bash
set -uo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
ARENA_DEBUG_SYNC=1 timeout -k 10 200 python scripts/debug_mimic_test.py > gpurun_out/mimic_eager.log 2>&1
echo "eager rc=$?"; grep -v "amdgpu.ids\|arena debug\] op" gpurun_out/mimic_eager.log | tail -5; grep "arena debug\] op" gpurun_out/mimic_eager.log | tail -2
ARENA_DEBUG_ALLOC=1 timeout -k 10 200 python scripts/debug_mimic_test.py > gpurun_out/mimic_graph.log 2>&1
echo "graph rc=$?"; grep -v "amdgpu.ids" gpurun_out/mimic_graph.log | tail -30
