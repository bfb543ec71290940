#!/bin/bash
# The committed-evidence run of a build (one gpurun call): smoke, the GPU
# suite, then the default bench under rocprofv3 --kernel-trace --stats (the
# bench line printed in the same run: scripts/trace_vs_bench.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
rm -rf gpurun_out/bench_trace gpurun_out/stages.log
bash scripts/gpu_check.sh tests || exit $?
grep -q "pytest_gpu rc=0" gpurun_out/stages.log || { echo "GPU suite failed"; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/bench_trace" -o run --output-format csv \
  -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_trace.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_trace.log | head -1 | cut -c1-300
