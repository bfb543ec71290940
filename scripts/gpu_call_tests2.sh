#!/bin/bash
# One gpurun call: the activation / K1 / DP tests changed this round, then
# the activation benches at cfg2's shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -q -p no:cacheprovider --timeout 240 --timeout-method thread tests/test_gpu_flow.py tests/test_gpu_rqs.py tests/test_gpu_train_dp.py -k "activation or kernel_selection or extremes_other or inverse_parity or fp32_kernel or two_lane or train_function or two_ranks" > gpurun_out/pt3.log 2>&1; echo "pytest rc=$?"; tail -8 gpurun_out/pt3.log
for c in cfg2sigmoid cfg2softplus cfg2relu; do
  timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-spline-kernel --no-configs > gpurun_out/b_$c.log 2>&1 || { tail -3 gpurun_out/b_$c.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/b_$c.log').read().strip().splitlines()[-1]); print('$c', round(d['value']/1e6,1), 'M/s', d['config'].get('kernel'), round(d['roofline']['kernel_us'],1), 'us')"
done
