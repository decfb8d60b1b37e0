#!/usr/bin/env bash
# Round 4: fp32 fused C3 (csrc/kernels/c3_x3.hip) — tests + engine A/B + op tables, then a short monolithic
# serving smoke (a server that fails to start shows its traceback in the arm log).
set -u
cd $GRAFT_REPO_ROOT
T=${1:-r4f}
bash scripts/gpurun/ab_engine.sh $T ARENA_FUSE_C3_F32 "0 1" "c3_x3 or fused_c3_program or pipeline_matches_reference or split_programs" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1 ARENA_NATIVE_HTTP=1 LOG_LEVEL=WARNING
timeout -k 10 400 python scripts/serving_sweep.py --archs monolithic --users 1,10 --procs 2 --warmup 2 --measure 8 \
  --cooldown 1 --runs 1 --out gpurun_out/$T/mono_smoke > gpurun_out/$T/mono_smoke.log 2>&1
echo "mono smoke rc=$?"
grep -h "users=" gpurun_out/$T/mono_smoke.log
for f in $(find gpurun_out/$T/mono_smoke -type f -size +2M); do tail -c 262144 "$f" > "$f.tail" && mv "$f.tail" "$f"; done
