#!/usr/bin/env bash
# GPU test suite, then the headline bench A/B of one executor knob on the same box.
# usage: AB_VAR=ARENA_STAGGER AB_VALS="0 0.25" [SKIP_TESTS=1] bash scripts/gpurun/r6_check.sh TAG
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=$1
O=gpurun_out/$T
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  $S 900 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
  grep -E "passed|failed" $O/pytest.log | tail -n 2 | tee -a $O/summary.txt
  grep -q " failed" $O/pytest.log && exit 1
fi
for v in ${AB_VALS:-}; do
  env ${AB_VAR}=$v $S 600 $O/bench_$v.log python -u bench.py --steps 20 --warmup 5 --latency-levels "" --no-secondary-inproc --no-secondary-bf16 || exit 1
  grep '^{' $O/bench_$v.log > $O/bench_$v.json
  python3 -c "import json,sys;d=json.load(open('$O/bench_$v.json'));print('$AB_VAR=$v', d['value'], d['p50_ms'], d['p99_ms'], d['engine_req_s'], d['engine_rgb_req_s'], d.get('gpu_busy'))" | tee -a $O/summary.txt
done
