#!/bin/bash
# End-of-milestone measurement in one gpurun call: rocprofv3 trace + PMC
# passes of the headline bench, the stall counters, every config, and the
# training-step throughput.  Each GPU step has its own time limit and the
# script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -rf gpurun_out/prof_* gpurun_out/pmc_st*
bash scripts/profile.sh || exit $?
bash scripts/pmc_stall.sh || exit $?
CONFIGS="cfg2 cfg3 cfg3s cfg4 cfg5 d8 cfg1" bash scripts/bench_configs.sh || exit $?
timeout -k 10 300 python scripts/train_bench.py > gpurun_out/train_bench.jsonl 2> gpurun_out/train_bench.err || exit $?
tail -9 gpurun_out/train_bench.jsonl
