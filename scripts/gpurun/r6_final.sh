#!/usr/bin/env bash
# Round-end tier as the driver runs it: the GPU test suite, smoke(), and the default bench.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=$1
O=gpurun_out/$T
mkdir -p $O
$S 900 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
grep -E "passed|failed" $O/pytest.log | tail -n 1 | tee -a $O/summary.txt
grep -q " failed" $O/pytest.log && exit 1
$S 300 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
tail -n 2 $O/smoke.log | tee -a $O/summary.txt
$S 900 $O/bench.log python -u bench.py || exit 1
grep '^{' $O/bench.log > $O/bench.json
python3 -c "import json;d=json.load(open('$O/bench.json'));print({k:d.get(k) for k in ['value','p50_ms','p99_ms','engine_req_s','engine_rgb_req_s','bs1_p50_ms','bs1_p99_ms','levels','gpu_busy']})" | tee -a $O/summary.txt
