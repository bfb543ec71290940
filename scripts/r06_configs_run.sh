#!/bin/bash
# Round-6 measurement call: every bench workload on one box (bench_configs.sh),
# stall counters of cfg3 / d8 / cfg5 (pmc_more_configs.sh), and three more
# headline runs for the box's spread.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
CONFIGS="cfg2 cfg3 cfg3s cfg4 cfg5 d8 d4k32 cfg1 cfg2relu cfg2gelu cfg2sigmoid cfg2softplus" bash scripts/bench_configs.sh || exit $?
bash scripts/pmc_more_configs.sh || exit $?
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-spline-kernel --no-configs > gpurun_out/rep_$r.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/rep_$r.log').read().strip().splitlines()[-1]); print('rep $r', round(d['value']/1e9,4), 'G/s', round(d['roofline']['kernel_us'],1), 'us', round(d['roofline']['frac'],4))" | tee -a gpurun_out/headline_reps.txt
done
