#!/bin/bash
# Every BASELINE config on one GPU (one gpurun call): one JSON line each into
# gpurun_out/configs.jsonl.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
: > gpurun_out/configs.jsonl
for c in ${CONFIGS:-cfg2 cfg3 cfg3s cfg4 cfg5}; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-spline-kernel > gpurun_out/cfg_$c.log 2>&1 || { tail -5 gpurun_out/cfg_$c.log; exit 1; }
  grep '^{' gpurun_out/cfg_$c.log >> gpurun_out/configs.jsonl
  python -c "import json,sys; d=json.loads(open('gpurun_out/cfg_$c.log').read().strip().splitlines()[-1]); print('$c', round(d['value']/1e6,1), 'M/s', round(d['roofline']['frac'],3), d.get('cpu_baseline',{}).get('value'))"
done
