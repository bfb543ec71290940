#!/bin/bash
# One gpurun call: smoke + the whole GPU suite (gpu_check.sh tests), then the
# stage-wise parity diagnostic of cfg4 (scripts/diag_stage.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_check.sh tests || exit $?
grep "pytest_gpu rc" gpurun_out/stages.log
timeout -k 10 300 python scripts/diag_stage.py cfg4 f16x2 > gpurun_out/diag_cfg4_f16x2.jsonl 2> gpurun_out/diag.err || { tail -5 gpurun_out/diag.err; exit 1; }
timeout -k 10 300 python scripts/diag_stage.py cfg4 fp32 > gpurun_out/diag_cfg4_fp32.jsonl 2>> gpurun_out/diag.err || { tail -5 gpurun_out/diag.err; exit 1; }
echo diag done
