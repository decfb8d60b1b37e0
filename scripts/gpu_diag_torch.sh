#!/usr/bin/env bash
set -uo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for m in eager recapture torch_first; do
  timeout -k 10 200 python scripts/debug_torch_big.py $m > gpurun_out/diag_$m.log 2>&1
  rc=$?
  grep -v amdgpu.ids gpurun_out/diag_$m.log | tail -4
  echo "$m rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
