#!/bin/bash
# bf16x3 training GEMM: parity tests, then train_bench A/B (ZF_TRAIN_X3=0/1)
# and a kernel-trace of the x3 run.
set -o pipefail
mkdir -p gpurun_out/tx3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 ./tune/gemm_probe > gpurun_out/tx3/probe.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train.py \
  -k "x3_gemm or 65536 or 32768" > gpurun_out/tx3/tests.txt 2>&1 &&
ZF_TRAIN_X3=0 timeout -k 10 300 python -u scripts/train_bench.py --configs cfg1,cfg2,cfg5 --batches 1024,65536 \
  > gpurun_out/tx3/bench_x3off.jsonl 2> gpurun_out/tx3/bench_x3off.err &&
ZF_TRAIN_X3=1 timeout -k 10 300 python -u scripts/train_bench.py --configs cfg1,cfg2,cfg5 --batches 1024,65536 \
  > gpurun_out/tx3/bench_x3on.jsonl 2> gpurun_out/tx3/bench_x3on.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tx3/prof -o run -- \
  python3 -u scripts/train_bench.py --configs cfg5 --batches 65536 --steps 10 > gpurun_out/tx3/prof.log 2>&1
