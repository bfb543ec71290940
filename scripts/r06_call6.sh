#!/bin/bash
# Round 6, sixth GPU call: the two-deep prefetch GEMM (training + layered
# parity), layered / training A/B against the previous commit's library, and
# a kernel trace of the new layered path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_dp.py tests/test_gpu_flow.py -m gpu -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread -k "train or layered or Layered or k100 or k200 or grad" > gpurun_out/c6_tests.log 2>&1
rc=$?; tail -3 gpurun_out/c6_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for v in gemm1 gemm2; do
  ZF_LIB=tune/lib$v.so timeout -k 10 300 python scripts/layered_bench.py --configs h512,h1024,h384c2 > gpurun_out/c6_layered_$v.jsonl 2> gpurun_out/c6_layered.err || { tail -5 gpurun_out/c6_layered.err; exit 1; }
  python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['config'], 'log_prob %.2f ms %.1f TF' % (d['log_prob']['ms'], d['log_prob']['tflops']), 'inverse %.2f ms' % d['inverse']['ms'])
" gpurun_out/c6_layered_$v.jsonl $v | tee -a gpurun_out/c6_layered_ab.txt
done; done
for v in gemm1 gemm2; do
  ZF_LIB=tune/lib$v.so timeout -k 10 300 python scripts/train_bench.py > gpurun_out/c6_train_$v.jsonl 2> gpurun_out/c6_train.err || exit $?
done
tail -9 gpurun_out/c6_train_gemm1.jsonl; tail -9 gpurun_out/c6_train_gemm2.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ZF_LIB=tune/libgemm2.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/c6_lay" -o run --output-format csv -- python3 scripts/layered_bench.py --configs h512 --rows 262144 --steps 3 > gpurun_out/c6_lay.log 2>&1 || { tail -5 gpurun_out/c6_lay.log; exit 1; }
echo done
