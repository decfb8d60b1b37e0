#!/usr/bin/env bash
# e2e HTTP rate vs decode processes / front-end threads (host-side budget of a 16-CPU share)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=${1:-decsweep}
mkdir -p gpurun_out/$T
for cfg in "10 4" "12 4" "12 2" "14 2" "13 3"; do
  set -- $cfg
  $S 240 gpurun_out/$T/w$1_t$2.log python bench.py --steps 30 --warmup 5 --no-secondary-bf16 --no-secondary-inproc --latency-levels "" --decode-workers $1 --http-threads $2 || exit 1
  echo "W=$1 T=$2: $(grep '"metric"' gpurun_out/$T/w$1_t$2.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_ms"], d["p99_ms"], d["engine_req_s"])')"
done
