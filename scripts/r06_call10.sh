#!/bin/bash
# Round 6: fused split-set combine — training suite with it on, bit identity
# against the two-launch form over 40 steps x 8 configs (twice), timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
ZF_TRAIN_FUSED_COMBINE=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_dp.py -m gpu -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/c10_tests.log 2>&1
rc=$?; tail -3 gpurun_out/c10_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/fused_combine_check.py gpurun_out/fc_plain.npz || exit $?
for r in 1 2; do
  ZF_TRAIN_FUSED_COMBINE=1 timeout -k 10 300 python scripts/fused_combine_check.py gpurun_out/fc_fused$r.npz || exit $?
  python scripts/fused_combine_check.py --compare gpurun_out/fc_fused$r.npz gpurun_out/fc_plain.npz | tee -a gpurun_out/c10_bits.txt
done
for r in 1 2; do for v in 0 1; do
  ZF_TRAIN_FUSED_COMBINE=$v timeout -k 10 200 python scripts/train_bench.py --configs cfg1,cfg2,cfg5 --batches 1024,4096 > gpurun_out/c10_train_$v.jsonl 2> gpurun_out/c10.err || { tail -3 gpurun_out/c10.err; exit 1; }
  sed "s/^/fused=$v /" gpurun_out/c10_train_$v.jsonl | tee -a gpurun_out/c10_train_ab.txt
done; done
rm -f gpurun_out/fc_*.npz
