#!/bin/bash
# Timing-only ablations: bench each zenflow_amd/variants/*.so (built with
# -DZF_X3_ABLATE=n) and print the fused kernel's average launch time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in zenflow_amd/variants/*.so; do
  ZF_LIB=$PWD/$v timeout -k 10 120 python bench.py --steps 20 --no-cpu-baseline --no-spline-kernel > gpurun_out/abl_run.log 2>&1 || { tail -5 gpurun_out/abl_run.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/abl_run.log').read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']/1e6,1), 'M/s', d['roofline']['kernel'])" "$v" | tee -a gpurun_out/abl.log
done
