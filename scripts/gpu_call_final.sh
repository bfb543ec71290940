#!/bin/bash
# Round-end check in one gpurun call: smoke, the whole GPU suite and the
# headline bench (gpu_check.sh all), then cfg5 / d8 / cfg4 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_check.sh all || exit $?
grep "pytest_gpu rc" gpurun_out/stages.log
CONFIGS="cfg5 d8 cfg4" bash scripts/bench_configs.sh || exit $?
