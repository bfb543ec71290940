#!/bin/bash
# One gpurun call: A/B of the pre-split dim-pair last layer (d8, cfg5), then
# the flow parity tests on that build (ZF_LIB).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
LIBS="pre0 pre1" ROUNDS=2 BENCH_ARGS="--config d8" STEPS=20 bash scripts/ab_libs.sh 2>&1 | tee gpurun_out/ab_pre_d8.txt || exit 1
LIBS="pre0 pre1" ROUNDS=2 BENCH_ARGS="--config cfg5" STEPS=10 bash scripts/ab_libs.sh 2>&1 | tee gpurun_out/ab_pre_cfg5.txt || exit 1
ZF_LIB=tune/libpre1.so timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 240 --timeout-method thread tests/test_gpu_flow.py tests/test_gpu_sampling.py > gpurun_out/pt_pre.log 2>&1; echo "pytest rc=$?"; tail -6 gpurun_out/pt_pre.log
