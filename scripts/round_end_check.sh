#!/bin/bash
# Round-end check in one gpurun call: smoke, the GPU suite and the headline
# bench (gpu_check.sh), the training-step sweep, and a rocprofv3 kernel
# trace of the K1 spline kernels (bench_rqs at the cfg2 coupling shape).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_check.sh all || exit $?
grep -q "rc=0" <(grep "pytest_gpu rc" gpurun_out/stages.log) || { echo "GPU suite failed"; exit 1; }
timeout -k 10 300 python scripts/train_bench.py > gpurun_out/train_bench.jsonl 2> gpurun_out/train_bench.err || exit $?
cat gpurun_out/train_bench.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/k1prof" -o run --output-format csv -- python3 scripts/bench_rqs.py 20 16 > gpurun_out/k1prof.log 2>&1 || exit $?
tail -1 gpurun_out/k1prof.log
