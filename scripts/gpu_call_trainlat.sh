#!/bin/bash
# Small-batch training step: split-set GEMM parity (fused combine, separate
# combine, single kernel), the gradient tests, then step latency for each
# form and a kernel trace of the cfg2 x 1024 step.
set -o pipefail
mkdir -p gpurun_out/tl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_train.py \
  > gpurun_out/tl/tests.txt 2>&1 || { tail -30 gpurun_out/tl/tests.txt; exit 1; }
tail -2 gpurun_out/tl/tests.txt
for r in 1 2; do
  for v in "1 1" "1 0" "0 1"; do
    set -- $v
    ZF_TRAIN_SPLITQ=$1 ZF_TRAIN_SPLITQ_FUSE=$2 timeout -k 10 120 python -u scripts/train_bench.py --configs cfg1,cfg2,cfg5 \
      --batches 1024 --steps 200 > gpurun_out/tl/sq$1f$2_r$r.jsonl 2> gpurun_out/tl/sq$1f$2.err || exit 1
    sed "s/^{/{\"splitq\": $1, \"fuse\": $2, /" gpurun_out/tl/sq$1f$2_r$r.jsonl
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/tl/prof -o run --output-format csv -- \
  python3 -u scripts/train_bench.py --configs cfg2 --batches 1024 --steps 50 > gpurun_out/tl/prof.log 2>&1
