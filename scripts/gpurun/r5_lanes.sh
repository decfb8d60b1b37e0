#!/usr/bin/env bash
# Head lanes root cause: the detector-only program behind the native batcher with lanes on (tools/lanes_repro.py,
# outside pytest so a fault leaves the native crash trace in its log), then the extended lanes GPU tests.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
O=gpurun_out/r5lanes
mkdir -p $O
$S 400 $O/repro_detector.log python -u tools/lanes_repro.py --program detector --users 1,2,10 --rounds 20 || { grep -A40 "arena crash" $O/repro_detector.log | head -60; exit 1; }
grep -A40 "arena crash" $O/repro_detector.log | head -60
grep -q "0 mismatches" $O/repro_detector.log || { tail -20 $O/repro_detector.log; exit 1; }
$S 400 $O/repro_export.log python -u tools/lanes_repro.py --program detector --users 2,10 --rounds 10 --export || { grep -A40 "arena crash" $O/repro_export.log | head -60; exit 1; }
$S 400 $O/repro_pipeline.log python -u tools/lanes_repro.py --program pipeline --users 1,2,10 --rounds 10 || { grep -A40 "arena crash" $O/repro_pipeline.log | head -60; exit 1; }
$S 600 $O/pytest.log python -u -m pytest tests/test_pipeline_gpu.py -k lanes -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
grep -E "passed|failed|error" $O/pytest.log | tail -3
