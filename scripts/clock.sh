#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"; REPO=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then L=""; else L="ZF_LIB=$REPO/zenflow_amd/variants/$v"; fi
  env $L timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d "$REPO/gpurun_out/clk_$v" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-spline-kernel > gpurun_out/clk_$v.log 2>&1 || exit $?
done
