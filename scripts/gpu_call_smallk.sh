#!/bin/bash
# First Dense at large batch on the one-thread-per-output kernel: gradient
# parity at the large-batch shapes, then the training throughput.
set -o pipefail
mkdir -p gpurun_out/sk
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_train_dp.py \
  > gpurun_out/sk/tests.txt 2>&1 || { tail -30 gpurun_out/sk/tests.txt; exit 1; }
tail -1 gpurun_out/sk/tests.txt
timeout -k 10 200 python -u scripts/train_bench.py --configs cfg1,cfg2,cfg5 --batches 1024,65536 > gpurun_out/sk/bench.jsonl 2>&1 || exit 1
cat gpurun_out/sk/bench.jsonl
