#!/usr/bin/env bash
# Closing check of HEAD after the head lanes went back to opt-in: the whole GPU tier, smoke() and the
# driver-shaped bench (the round-end driver runs the same three).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=r4closing2
mkdir -p gpurun_out/$T
$S 900 gpurun_out/$T/pytest.log python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider || exit 1
tail -2 gpurun_out/$T/pytest.log
grep -q " failed" gpurun_out/$T/pytest.log && exit 1
$S 300 gpurun_out/$T/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
tail -1 gpurun_out/$T/smoke.log
$S 600 gpurun_out/$T/bench.log python -u bench.py --steps 20 --warmup 5 || exit 1
grep '^{' gpurun_out/$T/bench.log | cut -c1-200
