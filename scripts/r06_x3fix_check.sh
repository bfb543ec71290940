#!/bin/bash
# Branch-free GEMM staging: full GPU suite, layered bench (bf16x3 and f16x2),
# training bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/x3fix_tests.log 2>&1; rc=$?; tail -3 gpurun_out/x3fix_tests.log; [ $rc -eq 0 ] || exit $rc
ZF_LAYERED_H2=0 timeout -k 10 300 python scripts/layered_bench.py --configs h512,h1024,h384c2 > gpurun_out/x3fix_lay_off.jsonl &&
timeout -k 10 300 python scripts/layered_bench.py --configs h512,h1024,h384c2 > gpurun_out/x3fix_lay_on.jsonl &&
cat gpurun_out/x3fix_lay_off.jsonl gpurun_out/x3fix_lay_on.jsonl &&
timeout -k 10 300 python scripts/train_bench.py --configs cfg1,cfg2,cfg5 > gpurun_out/x3fix_train.jsonl && cat gpurun_out/x3fix_train.jsonl
