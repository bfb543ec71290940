#!/bin/bash
# Small-batch training step after the launch merges: the training tests
# (bitwise DP / split-set / graph tests included), then step latency and a
# kernel trace of the cfg2 x 1024 step.
set -o pipefail
mkdir -p gpurun_out/tl2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py \
  tests/test_gpu_train_dp.py > gpurun_out/tl2/tests.txt 2>&1 || { tail -40 gpurun_out/tl2/tests.txt; exit 1; }
tail -2 gpurun_out/tl2/tests.txt
timeout -k 10 200 python -u scripts/train_bench.py --configs cfg1,cfg2,cfg5 --batches 1024,65536 --steps 200 \
  > gpurun_out/tl2/bench.jsonl 2> gpurun_out/tl2/bench.err || exit 1
cat gpurun_out/tl2/bench.jsonl
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/tl2/prof -o run --output-format csv -- \
  python3 -u scripts/train_bench.py --configs cfg2 --batches 1024 --steps 50 > gpurun_out/tl2/prof.log 2>&1
