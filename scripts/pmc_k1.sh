#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; REPO=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d "$REPO/gpurun_out/pmc$i" -o run --output-format csv -- python3 scripts/bench_rqs.py > gpurun_out/pmc$i.log 2>&1 || exit $?
done
timeout -k 10 120 python3 scripts/bench_rqs.py > gpurun_out/k1.log 2>&1
exit 0
