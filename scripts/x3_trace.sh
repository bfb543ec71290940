#!/bin/bash
# Build a ZF_X3_TRACE library and print the phase timing (one gpurun call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in ${VARIANTS:-0}; do
  ZF_LIB=$PWD/ab/libtrace.so timeout -k 10 200 python scripts/x3_trace.py > gpurun_out/trace_$v.log 2>&1 || { tail -20 gpurun_out/trace_$v.log; exit 1; }
done
