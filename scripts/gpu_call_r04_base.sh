#!/bin/bash
# Round-4 baseline in one gpurun call: rocprofv3 kernel trace of the exact
# bench invocation (its bench line in the same log), stall counters of the
# cfg4 / cfg3 / d8 instantiations, and the strict-parity GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; REPO=$(pwd); mkdir -p gpurun_out/r04
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$REPO/gpurun_out/r04/bench_trace" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/r04/bench_trace.log 2>&1 || { tail -5 gpurun_out/r04/bench_trace.log; exit 1; }
grep '^{' gpurun_out/r04/bench_trace.log | cut -c1-300
for c in cfg4 cfg3 d8; do
  PMC_PREFIX=r04/pmc_${c}_ BENCH_ARGS="--config $c" bash scripts/pmc_stall.sh || exit 1
done
rm -f gpurun_out/strict_parity.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_flow.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "strict or trained" > gpurun_out/r04/strict.log 2>&1; echo "strict rc=$?"; tail -3 gpurun_out/r04/strict.log
