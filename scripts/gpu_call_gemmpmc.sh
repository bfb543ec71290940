#!/bin/bash
# Counter passes over tests/hip/gemm_probe (tune/gemm_probe): the trainer's
# large-batch GEMM kernels.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/gp
run() { local name=$1; shift; timeout -s KILL 90 "$@" > "gpurun_out/gp/$name.log" 2>&1; local rc=$?; [ $rc -eq 0 ] || { tail -5 "gpurun_out/gp/$name.log"; exit $rc; }; }
run p1 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/gp/p1 -o run --output-format csv -- ./tune/gemm_probe
run p2 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/gp/p2 -o run --output-format csv -- ./tune/gemm_probe
run p3 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/gp/p3 -o run --output-format csv -- ./tune/gemm_probe
run p4 rocprofv3 --pmc WRITE_SIZE TCP_TCC_READ_REQ_sum --kernel-trace -d gpurun_out/gp/p4 -o run --output-format csv -- ./tune/gemm_probe
