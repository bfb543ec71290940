#!/bin/bash
# One gpurun call: A/B of the slot schedule on dim-pair flows' hidden layers
# (d8), then the flow parity tests on that build (ZF_LIB).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
LIBS="pp0 pp1" ROUNDS=2 BENCH_ARGS="--config d8" STEPS=20 bash scripts/ab_libs.sh 2>&1 | tee gpurun_out/ab_pairs.txt || exit 1
ZF_LIB=tune/libpp1.so timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 240 --timeout-method thread tests/test_gpu_flow.py tests/test_gpu_sampling.py > gpurun_out/pt_pairs.log 2>&1; echo "pytest rc=$?"; tail -6 gpurun_out/pt_pairs.log
