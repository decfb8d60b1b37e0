#!/usr/bin/env bash
# Host-memory retention: HIP-only repro modes (csrc/tests/hip_retention_repro.cpp), then the full GPU serving path
# (tools/leak_probe.py --gpu) per environment configuration ('+' separates assignments; "-" = defaults).
# usage: MODES="pack pack_same" bash scripts/gpurun/r6_leak.sh TAG - ARENA_STAGGER=0 ...
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
S=scripts/gpurun/gpu_step.sh
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
for m in ${MODES:-}; do
  $S 240 $O/repro_$m.log tools/bin/hip_retention_repro $m 6000 32 || exit 1
  tail -n 2 $O/repro_$m.log | head -n 1 | tee -a $O/summary.txt
done
i=0
for cfg in "$@"; do
  i=$((i + 1))
  envs=$(echo "$cfg" | tr '+' ' ')
  [ "$cfg" = "-" ] && envs="ARENA_X=0"
  env $envs $S ${STEP_S:-400} $O/srv_$i.log python -u tools/leak_probe.py --gpu --rounds ${ROUNDS:-6} --per-round ${PER:-30000} --users 64 ${LP_ARGS:-} || exit 1
  echo "[$cfg]" | tee -a $O/summary.txt
  grep "^round" $O/srv_$i.log | tee -a $O/summary.txt
done
