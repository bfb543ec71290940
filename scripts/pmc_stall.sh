#!/bin/bash
# Stall / co-execution counters of the fused kernel (two --pmc passes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
B=${PMC_CMD:-"python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-spline-kernel ${BENCH_ARGS:-}"}
P=${PMC_PREFIX:-pmc_st}
run() { local name=$1; shift; echo "=== $name"; timeout -s KILL 120 "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -2 "gpurun_out/$name.log"; [ $rc -eq 0 ] || exit $rc; }
run ${P}1 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d "$REPO/gpurun_out/${P}1" -o run --output-format csv -- $B
run ${P}2 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d "$REPO/gpurun_out/${P}2" -o run --output-format csv -- $B
run ${P}3 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_INST_LEVEL_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAVES SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --kernel-trace -d "$REPO/gpurun_out/${P}3" -o run --output-format csv -- $B
