#!/bin/bash
# Round 6: K1 K=16 occupancy A/B (register-allocator wave targets 4 / 6 / 8).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
ZF_LIB=tune/libk1w8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_rqs.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/c8_tests.log 2>&1
rc=$?; tail -2 gpurun_out/c8_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do LIBS="k1w0 k1w6 k1w8" KS="16" bash scripts/ab_rqs.sh | tee -a gpurun_out/c8_k1_ab.txt || exit $?; done
