#!/bin/bash
# Trainer fp32 MFMA GEMM with store-time masking (in-tree) vs select-after-load
# (tune/libmg0.so): GPU suite, then the training bench interleaved, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/mg_tests.log 2>&1; rc=$?; tail -2 gpurun_out/mg_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  echo "== before"; ZF_LIB=tune/libmg0.so timeout -k 10 300 python scripts/train_bench.py --configs cfg1,cfg2,cfg5 || exit $?
  echo "== after"; timeout -k 10 300 python scripts/train_bench.py --configs cfg1,cfg2,cfg5 || exit $?
done
