#!/usr/bin/env bash
# the round-end GPU tier: pytest -m gpu (one process), then smoke(); usage: scripts/gpurun/gputests.sh TAG [pytest -k expr]
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-gputests}
K=${2:-}
mkdir -p gpurun_out/$T
if [ -n "$K" ]; then
  $S 1000 gpurun_out/$T/pytest.log python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 180 --timeout-method thread -p no:cacheprovider || exit 1
else
  $S 1000 gpurun_out/$T/pytest.log python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider || exit 1
fi
tail -15 gpurun_out/$T/pytest.log
$S 300 gpurun_out/$T/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
tail -3 gpurun_out/$T/smoke.log
