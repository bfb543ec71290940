#!/bin/bash
# Stall counters of the two-set kernel (cfg2) beside flow_kernel_x3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/x4
export HSA_ENABLE_IPC_MODE_LEGACY=0
for c in ${CFGS:-cfg2}; do
  ZF_X4=1 PMC_PREFIX=x4/pmc4_${c}_ BENCH_ARGS="--config $c" bash scripts/pmc_stall.sh || exit 1
  ZF_X4=0 PMC_PREFIX=x4/pmc3_${c}_ BENCH_ARGS="--config $c" bash scripts/pmc_stall.sh || exit 1
done
