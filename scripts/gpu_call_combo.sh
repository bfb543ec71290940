#!/bin/bash
# x4 ablations + targeted parity of the changed x3 paths + benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/x4
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_call_x4abl.sh || exit 1
rm -f gpurun_out/acts_tiny.jsonl
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 240 --timeout-method thread tests/test_gpu_flow.py -k "other_acts or (log_prob_parity and (cfg4 or cfg1 or d3c1 or k5c1 or softplus or sigmoid)) or kernel_selection or trained or strict" > gpurun_out/x4/pt_combo.log 2>&1
rc=$?; tail -4 gpurun_out/x4/pt_combo.log; cat gpurun_out/acts_tiny.jsonl 2>/dev/null
for c in cfg4 cfg2softplus cfg2sigmoid cfg2relu; do
  ZF_X4=0 timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-spline-kernel > gpurun_out/x4/c_$c.log 2>&1 || { tail -3 gpurun_out/x4/c_$c.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/x4/c_$c.log') if l.startswith('{')][-1]); print('$c', round(d['value']/1e6,1), 'M/s', round(d['roofline']['frac'],3), d['config'].get('kernel'))"
done
