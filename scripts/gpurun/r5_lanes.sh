#!/usr/bin/env bash
# Head lanes: the detector-only program behind the native batcher with lanes on under the arm-B services' queue
# cap (GPU_MAX_HW_QUEUES=2: the configuration that segfaulted inside hipGraphLaunch of the forked graph), outside
# pytest so a fault leaves the native crash trace in its log; then the extended lanes GPU tests and a bs-1 / bs-2
# latency A/B of the fused pipeline (lanes off vs on, queues 4).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
O=gpurun_out/r5lanes
mkdir -p $O
crash() { grep -m1 -A12 "arena crash" $1 | head -14; exit 1; }
GPU_MAX_HW_QUEUES=2 $S 400 $O/repro_detector_q2.log python -u tools/lanes_repro.py --program detector --users 1,2,10 --rounds 40 || crash $O/repro_detector_q2.log
grep -q "0 mismatches" $O/repro_detector_q2.log || { tail -20 $O/repro_detector_q2.log; exit 1; }
GPU_MAX_HW_QUEUES=1 $S 400 $O/repro_detector_q1.log python -u tools/lanes_repro.py --program detector --users 1,2,10 --rounds 20 --export || crash $O/repro_detector_q1.log
grep -q "0 mismatches" $O/repro_detector_q1.log || { tail -20 $O/repro_detector_q1.log; exit 1; }
$S 600 $O/pytest.log python -u -m pytest tests/test_pipeline_gpu.py -k lanes -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
grep -E "passed|failed|error" $O/pytest.log | tail -3
grep -q " failed\| error" $O/pytest.log && exit 1
$S 400 $O/latency_pipeline.log python -u tools/lanes_repro.py --program pipeline --users 1,2 --rounds 400 || crash $O/latency_pipeline.log
grep "round latency\|mismatches" $O/latency_pipeline.log
