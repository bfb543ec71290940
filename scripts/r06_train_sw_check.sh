#!/bin/bash
# Trainer GEMMs with swish-only epilogue instantiations: full GPU suite, training bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/trsw_tests.log 2>&1; rc=$?; tail -3 gpurun_out/trsw_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/train_bench.py --configs cfg1,cfg2,cfg5 > gpurun_out/trsw_train.jsonl && cat gpurun_out/trsw_train.jsonl
