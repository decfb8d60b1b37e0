#!/usr/bin/env bash
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x -k "${PYTEST_K:-ir_block or pipeline}" > gpurun_out/pytest_iter.log 2>&1 || { tail -60 gpurun_out/pytest_iter.log; exit 1; }
tail -1 gpurun_out/pytest_iter.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/bench.json 2> gpurun_out/bench.err
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print('bench', d['value'], d['p50_ms'], d['bs1_p50_ms'])"
if [ "${SWEEP:-1}" = "1" ]; then
  timeout -k 10 900 python scripts/serving_sweep.py --archs ${ARCHS:-monolithic,triton,microservices} --users ${USERS:-1,10,50,100} \
    --warmup 5 --measure 15 --procs 4 --procs-per-gpu ${PPG:-4} --out gpurun_out/load 2>&1 | grep -v amdgpu.ids | tee gpurun_out/load_sweep.log
fi
