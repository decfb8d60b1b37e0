#!/usr/bin/env bash
# Round 4: the split JPEG decoder on the GPU (kernel + executor + front-end tests), smoke, then the driver's
# bench.  usage: scripts/gpurun/r4_check.sh TAG [extra pytest targets] -- [bench args]
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-r4}
shift
TESTS=""
while [ $# -gt 0 ] && [ "$1" != "--" ]; do TESTS="$TESTS $1"; shift; done
[ $# -gt 0 ] && shift
mkdir -p gpurun_out/$T
if [ -n "$TESTS" ]; then
  $S 900 gpurun_out/$T/pytest.log python -u -m pytest $TESTS -x -v --timeout 180 --timeout-method thread -p no:cacheprovider || exit 1
  grep -E "passed|failed|error" gpurun_out/$T/pytest.log | tail -3
  grep -q " failed\| error" gpurun_out/$T/pytest.log && exit 1
fi
$S 300 gpurun_out/$T/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S 900 gpurun_out/$T/bench.log python -u bench.py "$@" || exit 1
grep '^{' gpurun_out/$T/bench.log | tail -1 > gpurun_out/$T/bench.json
cut -c1-1500 gpurun_out/$T/bench.json
