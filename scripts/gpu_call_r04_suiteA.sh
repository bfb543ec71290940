#!/bin/bash
# Round-4 final, part A: the whole GPU suite (no -x: failures are recorded),
# then the layered-path and training throughput lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r04f
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
rm -f gpurun_out/strict_parity.jsonl gpurun_out/acts_tiny.jsonl gpurun_out/grad_parity.jsonl
timeout -k 10 960 python -u -m pytest -q -p no:cacheprovider --timeout 240 --timeout-method thread tests -m gpu > gpurun_out/r04f/suite.log 2>&1
rc=$?; tail -3 gpurun_out/r04f/suite.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 120 python -u scripts/layered_bench.py --configs h512,h1024,h384c2 > gpurun_out/r04f/layered_bench.jsonl 2> gpurun_out/r04f/layered_bench.err || exit 1
cat gpurun_out/r04f/layered_bench.jsonl
exit $rc
