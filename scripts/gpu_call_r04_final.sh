#!/bin/bash
# Round-4 final measurement in one gpurun call: the GPU suite, the exact
# bench invocation under rocprofv3 (trace vs bench line), stall counters of
# every headline instantiation, FETCH/WRITE traffic, every config.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; REPO=$(pwd); mkdir -p gpurun_out/r04f
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
rm -f gpurun_out/strict_parity.jsonl gpurun_out/acts_tiny.jsonl
if [ -z "${SKIP_SUITE:-}" ]; then
  # the whole suite (no -x: a failing test is recorded, the measurements still run)
  timeout -k 10 1000 python -u -m pytest -q -p no:cacheprovider --timeout 240 --timeout-method thread tests -m gpu > gpurun_out/r04f/suite.log 2>&1
  rc=$?; tail -3 gpurun_out/r04f/suite.log
  # only a timeout, abort or crash stops the call (no GPU work after a fault)
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$REPO/gpurun_out/r04f/bench_trace" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/r04f/bench_trace.log 2>&1 || { tail -5 gpurun_out/r04f/bench_trace.log; exit 1; }
grep '^{' gpurun_out/r04f/bench_trace.log | cut -c1-200
for c in ${PMC_CONFIGS:-cfg2 cfg4 cfg3 d8}; do
  PMC_PREFIX=r04f/pmc_${c}_ BENCH_ARGS="--config $c" bash scripts/pmc_stall.sh || exit 1
done
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-spline-kernel"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$REPO/gpurun_out/r04f/prof_fetch" -o run --output-format csv -- $B > gpurun_out/r04f/prof_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$REPO/gpurun_out/r04f/prof_write" -o run --output-format csv -- $B > gpurun_out/r04f/prof_write.log 2>&1 || exit 1
CONFIGS="${CONFIGS:-cfg2 cfg3 cfg3s cfg4 cfg5 d8 cfg1 cfg2sigmoid cfg2softplus cfg2relu}" bash scripts/bench_configs.sh || exit 1
cp gpurun_out/configs.jsonl gpurun_out/r04f/configs.jsonl

timeout -k 10 300 python -u scripts/train_bench.py --configs cfg1,cfg2,cfg5 --batches 1024,65536 > gpurun_out/r04f/train_bench.jsonl 2> gpurun_out/r04f/train_bench.err || exit 1
