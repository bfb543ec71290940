#!/bin/bash
# Round 6, fifth GPU call: layered path + training suites after the small-K
# and WIDE-epilogue changes, layered bench + kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_dp.py tests/test_gpu_flow.py -m gpu -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread -k "train or layered or Layered or k100 or k200 or grad" > gpurun_out/c5_tests.log 2>&1
rc=$?; tail -3 gpurun_out/c5_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/layered_bench.py --configs h512,h1024,h384c2 > gpurun_out/c5_layered.jsonl 2> gpurun_out/c5_layered.err || { tail -5 gpurun_out/c5_layered.err; exit 1; }
cat gpurun_out/c5_layered.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/c5_lay" -o run --output-format csv -- python3 scripts/layered_bench.py --configs h512 --rows 262144 --steps 3 > gpurun_out/c5_lay.log 2>&1 || { tail -5 gpurun_out/c5_lay.log; exit 1; }
timeout -k 10 300 python scripts/train_bench.py > gpurun_out/c5_train_bench.jsonl 2> gpurun_out/c5_train_bench.err || exit $?
cat gpurun_out/c5_train_bench.jsonl
