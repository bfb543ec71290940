#!/bin/bash
# Round 6: small-batch training step with and without the split-set GEMMs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2; do for v in 1 0; do
  ZF_TRAIN_SPLITQ=$v timeout -k 10 200 python scripts/train_bench.py --configs cfg1,cfg2,cfg5 --batches 1024,4096 > gpurun_out/c9_train_$v.jsonl 2> gpurun_out/c9.err || { tail -3 gpurun_out/c9.err; exit 1; }
  sed "s/^/splitq=$v /" gpurun_out/c9_train_$v.jsonl | tee -a gpurun_out/c9_train_ab.txt
done; done
