#!/bin/bash
# Training step with the split-set small GEMMs (default) vs one launch per
# GEMM (ZF_TRAIN_SPLITQ=0): same bits, fewer launches; two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2; do
  echo "== split"; timeout -k 10 200 python scripts/train_bench.py --configs cfg1,cfg2,cfg5 --batches 1024,4096,16384 || exit $?
  echo "== nosplit"; ZF_TRAIN_SPLITQ=0 timeout -k 10 200 python scripts/train_bench.py --configs cfg1,cfg2,cfg5 --batches 1024,4096,16384 || exit $?
done
