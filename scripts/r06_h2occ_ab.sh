#!/bin/bash
# gemm_h2_kernel: two blocks per CU with the double-buffered stage (in-tree)
# vs three with the single-buffer stage (tune/libh2occ3.so, spills 10-15
# VGPRs on the swish forms), three interleaved rounds, after its parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
ZF_LIB=tune/libh2occ3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_flow.py -x -q --timeout 120 --timeout-method thread -k "h512 or h384c2 or h1024k5 or h260 or layered" > gpurun_out/h2occ_tests.log 2>&1; rc=$?; tail -2 gpurun_out/h2occ_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  echo "== occ2"; timeout -k 10 200 python scripts/layered_bench.py --configs h512,h1024,h384c2 || exit $?
  echo "== occ3"; ZF_LIB=tune/libh2occ3.so timeout -k 10 200 python scripts/layered_bench.py --configs h512,h1024,h384c2 || exit $?
done
