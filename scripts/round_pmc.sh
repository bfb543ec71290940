#!/bin/bash
# Counter passes of a build (one gpurun call): the stall / pipe counters of
# the headline kernel (cfg2) and of cfg4 (scripts/pmc_stall.sh), and the HBM
# traffic passes (FETCH_SIZE / WRITE_SIZE) of the default bench.  Summaries:
# scripts/summarize_stall.py, scripts/summarize_profiles.py (CPU side).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc_st* gpurun_out/pmc_c4* gpurun_out/prof_fetch gpurun_out/prof_write
PMC_PREFIX=pmc_st bash scripts/pmc_stall.sh || exit $?
PMC_PREFIX=pmc_c4 BENCH_ARGS="--config cfg4" bash scripts/pmc_stall.sh || exit $?
REPO=$(pwd); B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-spline-kernel"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$REPO/gpurun_out/prof_fetch" -o run --output-format csv -- $B > gpurun_out/prof_fetch.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$REPO/gpurun_out/prof_write" -o run --output-format csv -- $B > gpurun_out/prof_write.log 2>&1 || exit $?
echo done
